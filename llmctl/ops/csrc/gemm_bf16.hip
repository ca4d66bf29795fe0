// bf16 MFMA GEMM  C[M,N] = A[M,K] · B[N,K]^T  (fp32 accumulate) + an HBM copy kernel (gfx950).
//
// Used by `llmctl hw benchmark --component compute`, `llmctl bench kernels --matmul` and the
// autotuner (projection GEMMs in training go to hipBLASLt through torch).  Structure
// (CDNA guide §5 "standard MFMA GEMM main loop"): 128x128 workgroup tile, 4 waves in a
// 2x2 grid each owning 64x64 (2x2 mfma_f32_32x32x16_bf16 accumulators), BK = 64, LDS double
// buffer filled by register staging (next tile's global loads issued before this tile's
// MFMAs, written after the barrier — T14), XOR-swizzled 128-B LDS rows so the 32 lanes of
// a ds_read_b128 hit distinct banks (T2), and an XCD-aware block remap so workgroups that
// share A/B panels run on the same XCD's L2 (T1).
#include "attn_common.h"

namespace llmctl {
using namespace attn;
namespace {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int ROWB = BK * 2;  // 128 bytes per LDS row

__device__ __forceinline__ int g_off(int row, int chunk) {  // swizzled LDS byte offset
  return row * ROWB + ((chunk ^ ((row >> 1) & 7)) << 4);
}

__global__ __launch_bounds__(256, 2) void gemm_nt_kernel(const unsigned short* __restrict__ A,
                                                          const unsigned short* __restrict__ B,
                                                          unsigned short* __restrict__ C, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * 2 * BM * ROWB];  // 2 buffers x (A,B)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = N / BN;
  const int nwg = gridDim.x;
  // XCD-aware bijective remap (guide §5: blocks b, b+8, ... share an XCD)
  const int bid = blockIdx.x;
  int wg = bid;
  if (nwg >= 8) {
    const int q = nwg / 8, rem = nwg % 8, x = bid % 8;
    wg = (x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q) + bid / 8;
  }
  const int tm = wg / tiles_n, tn = wg % tiles_n;
  const unsigned short* Ab = A + (long)tm * BM * K;
  const unsigned short* Bb = B + (long)tn * BN * K;

  uint4 sa[4], sb[4];
  auto issue = [&](int kt) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int c = tid + 256 * it;
      const int row = c >> 3, ch = c & 7;
      sa[it] = *reinterpret_cast<const uint4*>(Ab + (long)row * K + kt * BK + ch * 8);
      sb[it] = *reinterpret_cast<const uint4*>(Bb + (long)row * K + kt * BK + ch * 8);
    }
  };
  auto commit = [&](int buf) {
    unsigned char* As = smem + buf * 2 * BM * ROWB;
    unsigned char* Bs = As + BM * ROWB;
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int c = tid + 256 * it;
      const int row = c >> 3, ch = c & 7;
      *reinterpret_cast<uint4*>(As + g_off(row, ch)) = sa[it];
      *reinterpret_cast<uint4*>(Bs + g_off(row, ch)) = sb[it];
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int KT = K / BK;
  issue(0);
  commit(0);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < KT) issue(kt + 1);
    const unsigned char* As = smem + buf * 2 * BM * ROWB;
    const unsigned char* Bs = As + BM * ROWB;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8_t af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = lds_read_b128(As, g_off(wm * 64 + i * 32 + r, 2 * ks + h));
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = lds_read_b128(Bs, g_off(wn * 64 + j * 32 + r, 2 * ks + h));
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma32(af[i], bfr[j], acc[i][j]);
    }
    if (kt + 1 < KT) {
      commit(buf ^ 1);  // other buffer: last read one iteration ago (barrier below orders it)
    }
    __syncthreads();
  }
  // epilogue: reg e -> row acc_row(e, h), col = r
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = tn * BN + wn * 64 + j * 32 + r;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = tm * BM + wm * 64 + i * 32 + acc_row(e, h);
        C[(long)row * N + col] = f2bf(acc[i][j][e]);
      }
    }
}

__global__ __launch_bounds__(256) void copy_kernel(const uint4* __restrict__ s, uint4* __restrict__ d, long n16) {
  const long stride = (long)gridDim.x * 256;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) d[i] = s[i];
}

}  // namespace

at::Tensor gemm_bf16(const at::Tensor& a, const at::Tensor& b) {
  LLMCTL_CHECK(a.dim() == 2 && b.dim() == 2 && a.is_contiguous() && b.is_contiguous() &&
                   a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16,
               "gemm_bf16: contiguous bf16 A[M,K], B[N,K]");
  const int M = a.size(0), K = a.size(1), N = b.size(0);
  LLMCTL_CHECK(b.size(1) == K, "gemm_bf16: K mismatch");
  LLMCTL_CHECK(M % BM == 0 && N % BN == 0 && K % BK == 0, "gemm_bf16: M,N multiple of 128 and K of 64");
  const c10::DeviceGuard g(a.device());
  auto c = at::empty({M, N}, a.options());
  hipLaunchKernelGGL(gemm_nt_kernel, dim3((M / BM) * (N / BN)), dim3(256), 0, stream(), bf_ptr(a), bf_ptr(b),
                     bf_mut(c), M, N, K);
  return c;
}

void hbm_copy(const at::Tensor& src, at::Tensor& dst) {
  LLMCTL_CHECK(src.is_contiguous() && dst.is_contiguous() && src.nbytes() == dst.nbytes() && src.nbytes() % 16 == 0,
               "hbm_copy: contiguous, equal size, multiple of 16 bytes");
  const c10::DeviceGuard g(src.device());
  const long n16 = src.nbytes() / 16;
  const int grid = (int)std::min<long>((n16 + 255) / 256, (long)num_cus() * 8);
  hipLaunchKernelGGL(copy_kernel, dim3(grid), dim3(256), 0, stream(), reinterpret_cast<const uint4*>(src.data_ptr()),
                     reinterpret_cast<uint4*>(dst.data_ptr()), n16);
}

TORCH_LIBRARY_IMPL(llmctl, CUDA, m) {
  m.impl("gemm_bf16", &gemm_bf16);
  m.impl("hbm_copy", &hbm_copy);
}

}  // namespace llmctl
