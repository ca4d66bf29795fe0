// bf16 matrix transpose dst[C][R] = src[R][C] (gfx950), for the transposed weight copies the
// data-gradient GEMMs read (llmctl.exec.linear: dX = dY W runs as F.linear(dY, W^T) — the
// forward's layout, ~13 % faster on hipBLASLt than dY @ W; profiles/gemm_tunable_dgradT_r1.log).
//
// 64x64 tiles per 256-thread workgroup: 16-B row loads (a wave covers 8 rows x 128 B), the tile
// is written transposed into LDS with 2-B stores (row stride 144 B: the 8 lanes of a store that
// share an LDS row hit distinct banks), then read back as 16-B rows and stored coalesced.
// Memory-bound: ~2 x 8 KB of HBM traffic per tile.
#include "common.h"

namespace llmctl {
namespace {

constexpr int TT = 64;          // tile edge
constexpr int LROW = TT + 8;    // LDS row (elements): 144 B, keeps 16-B alignment

__global__ __launch_bounds__(256) void transpose_bf16_kernel(const unsigned short* __restrict__ src,
                                                             unsigned short* __restrict__ dst, int R, int C,
                                                             int tiles_c) {
  __shared__ __attribute__((aligned(16))) unsigned short t[TT * LROW];
  const int tr = blockIdx.x / tiles_c, tc = blockIdx.x % tiles_c;
  const int r0 = tr * TT, c0 = tc * TT;
  const int tid = threadIdx.x;
  const int ch = tid & 7;    // 16-B chunk within a 64-element row
  const int rr = tid >> 3;   // 0..31
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int r = rr + 32 * it;
    const int gr = r0 + r, gc = c0 + ch * 8;
    bf16x8 v{};
    if (gr < R && gc < C) v = *reinterpret_cast<const bf16x8*>(src + (size_t)gr * C + gc);
#pragma unroll
    for (int j = 0; j < 8; ++j) t[(ch * 8 + j) * LROW + r] = v[j];
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int c = rr + 32 * it;  // output row = source column
    const int gc = c0 + c, gr = r0 + ch * 8;
    if (gc < C && gr < R)
      *reinterpret_cast<bf16x8*>(dst + (size_t)gc * R + gr) = *reinterpret_cast<const bf16x8*>(&t[c * LROW + ch * 8]);
  }
}

}  // namespace

void transpose_(const at::Tensor& src, at::Tensor& dst) {
  LLMCTL_CHECK(src.is_cuda() && dst.is_cuda() && src.dim() == 2 && dst.dim() == 2, "transpose_: 2-D GPU tensors");
  LLMCTL_CHECK(src.scalar_type() == at::kBFloat16 && dst.scalar_type() == at::kBFloat16, "transpose_: bf16");
  LLMCTL_CHECK(src.is_contiguous() && dst.is_contiguous(), "transpose_: contiguous");
  const long R = src.size(0), C = src.size(1);
  LLMCTL_CHECK(dst.size(0) == C && dst.size(1) == R, "transpose_: dst must be [C, R]");
  LLMCTL_CHECK(R % 8 == 0 && C % 8 == 0, "transpose_: dims must be multiples of 8");
  LLMCTL_CHECK((reinterpret_cast<uintptr_t>(src.data_ptr()) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(dst.data_ptr()) & 15) == 0,
               "transpose_: 16-B aligned");
  if (R == 0 || C == 0) return;
  const c10::DeviceGuard g(src.device());
  const int tiles_r = (R + TT - 1) / TT, tiles_c = (C + TT - 1) / TT;
  hipLaunchKernelGGL(transpose_bf16_kernel, dim3((unsigned)(tiles_r * tiles_c)), dim3(256), 0, stream(),
                     bf_ptr(src), bf_mut(dst), (int)R, (int)C, tiles_c);
}

TORCH_LIBRARY_IMPL(llmctl, CUDA, m) { m.impl("transpose_", &transpose_); }

}  // namespace llmctl
