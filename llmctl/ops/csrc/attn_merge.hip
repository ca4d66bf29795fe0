// Log-sum-exp merge of partial attention outputs (ring / context-parallel attention), gfx950.
//
//   lse' = logaddexp(lse_acc, lse_j)
//   o'   = o_acc * exp(lse_acc - lse') + o_j * exp(lse_j - lse')
//
// o_acc fp32 [B,S,H,D] and lse_acc fp32 [B,H,S] are updated in place; o_j is the bf16 output
// of one flash-attention call ([B,S,H,D], any row strides) with its natural-log LSE lse_j.  A
// fresh accumulator is o_acc = 0, lse_acc = -inf.  Rows where both LSEs are -inf (no visible
// key yet) stay 0 / -inf.  One pass over the partial instead of ~10 fp32 torch elementwise
// kernels (the eager merge of round 1).  Lanes: D/8 per (b, s, h) row, 8 elements each.
#include "common.h"

namespace llmctl {
namespace {

template <int D>
__global__ __launch_bounds__(256) void attn_merge_kernel(float* __restrict__ o_acc, float* __restrict__ lse_acc,
                                                         const unsigned short* __restrict__ o_j,
                                                         const float* __restrict__ lse_j, int B, int S, int H,
                                                         long j_sb, long j_ss, long j_sh) {
  constexpr int LPR = D / 8;
  const long gid = (long)blockIdx.x * 256 + threadIdx.x;
  const long row = gid / LPR;  // (b, s, h)
  const int sub = gid % LPR;
  if (row >= (long)B * S * H) return;
  const int h = row % H;
  const long bs = row / H;
  const int s = bs % S;
  const int b = bs / S;
  const long li = ((long)b * H + h) * S + s;
  const float la = lse_acc[li], lj = lse_j[li];
  const float m = fmaxf(la, lj);
  float wa = 0.f, wj = 0.f, ln = -INFINITY;
  if (m != -INFINITY) {
    const float ea = __expf(la - m), ej = __expf(lj - m);
    ln = m + __logf(ea + ej);
    wa = ea / (ea + ej);
    wj = ej / (ea + ej);
  }
  float* po = o_acc + row * D + sub * 8;
  float x[8], y[8];
#pragma unroll
  for (int k = 0; k < 8; k += 4) {
    const float4 t = *reinterpret_cast<const float4*>(po + k);
    x[k] = t.x;
    x[k + 1] = t.y;
    x[k + 2] = t.z;
    x[k + 3] = t.w;
  }
  load8(o_j + b * j_sb + (long)s * j_ss + (long)h * j_sh + sub * 8, y);
#pragma unroll
  for (int k = 0; k < 8; k += 4)
    *reinterpret_cast<float4*>(po + k) = make_float4(wa * x[k] + wj * y[k], wa * x[k + 1] + wj * y[k + 1],
                                                     wa * x[k + 2] + wj * y[k + 2], wa * x[k + 3] + wj * y[k + 3]);
  if (sub == 0) lse_acc[li] = ln;
}

}  // namespace

void attn_merge_(at::Tensor& o_acc, at::Tensor& lse_acc, const at::Tensor& o_j, const at::Tensor& lse_j) {
  LLMCTL_CHECK(o_acc.dim() == 4 && o_acc.scalar_type() == at::kFloat && o_acc.is_contiguous(),
               "attn_merge_: o_acc fp32 contiguous [B,S,H,D]");
  const int B = o_acc.size(0), S = o_acc.size(1), H = o_acc.size(2), D = o_acc.size(3);
  LLMCTL_CHECK(D == 64 || D == 128, "attn_merge_: head_dim 64 or 128");
  LLMCTL_CHECK(o_j.sizes() == o_acc.sizes() && o_j.scalar_type() == at::kBFloat16 && o_j.stride(3) == 1 &&
                   o_j.stride(0) % 8 == 0 && o_j.stride(1) % 8 == 0 && o_j.stride(2) % 8 == 0 &&
                   (reinterpret_cast<uintptr_t>(o_j.data_ptr()) & 15) == 0,
               "attn_merge_: o_j bf16 [B,S,H,D], 16-B aligned rows");
  for (const at::Tensor* t : {static_cast<const at::Tensor*>(&lse_acc), &lse_j})
    LLMCTL_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == (long)B * H * S,
                 "attn_merge_: lse fp32 contiguous [B,H,S]");
  if ((long)B * S * H == 0) return;
  const c10::DeviceGuard g(o_acc.device());
  const long threads = (long)B * S * H * (D / 8);
  const dim3 grid((unsigned)((threads + 255) / 256));
  if (D == 128)
    hipLaunchKernelGGL(attn_merge_kernel<128>, grid, dim3(256), 0, stream(), o_acc.data_ptr<float>(),
                       lse_acc.data_ptr<float>(), reinterpret_cast<const unsigned short*>(o_j.data_ptr()),
                       lse_j.data_ptr<float>(), B, S, H, o_j.stride(0), o_j.stride(1), o_j.stride(2));
  else
    hipLaunchKernelGGL(attn_merge_kernel<64>, grid, dim3(256), 0, stream(), o_acc.data_ptr<float>(),
                       lse_acc.data_ptr<float>(), reinterpret_cast<const unsigned short*>(o_j.data_ptr()),
                       lse_j.data_ptr<float>(), B, S, H, o_j.stride(0), o_j.stride(1), o_j.stride(2));
}

TORCH_LIBRARY_IMPL(llmctl, CUDA, m) { m.impl("attn_merge_", &attn_merge_); }

}  // namespace llmctl
