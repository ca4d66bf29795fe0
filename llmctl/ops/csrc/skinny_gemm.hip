// Decode-shaped GEMM (gfx950): y[M,N] = x[M,K] · W[N,K]^T (+ bias), M <= 32 tokens.
//
// A decode step reads every projection weight once for a handful of tokens: the op is an HBM
// stream of W (13 GB per GPT-7B step); hipBLASLt's small-M kernels reach 3.6-3.8 TB/s on the
// wide projections but only 1.8-2.4 TB/s on the 4096-row ones (too few workgroups).  Here:
//   * MFMA 16x16x32 bf16 with the WEIGHT rows on the MFMA row axis and the tokens on the
//     column axis: a wave owns 16 weight rows and MT x 16 token columns;
//   * the K reduction order is free, so the lane group g = lane/16 of MFMA step s reads real
//     k = kb + 32 g + 8 s + j: every lane streams 64 contiguous bytes of its weight row per
//     128-deep K block (4 dwordx4 loads), the token operand uses the same permutation;
//   * a workgroup = 8 waves on one 16-row tile, splitting K 8 ways; GB K blocks per wave are
//     loaded before the first MFMA (16-32 KB of weight loads in flight per wave, the whole
//     CU's share of the stream), the 8 partial tiles are reduced through LDS;
//   * grid = N/16 workgroups (256 for a 4096-row projection: one per CU).
// Measured (uncached weights, tools/decode_bench.py): 1.5-1.9x hipBLASLt on the narrow
// projections (o-proj, down-proj), slower than it on the wide ones at M >= 8, which is why
// ops.decode_linear routes only out_features <= 4096 here.
// Weights are read with plain loads (they are not reused within a step; the L2/MALL decides):
// non-temporal (nt) weight loads measured 30 % slower on every GPT-7B projection (qkv 35.4 vs
// 24.6 us, decode step 8.26 vs 6.87 ms; profiles/decode_gemm_nt_r5.txt).
#include <cstdlib>

#include "attn_common.h"

namespace llmctl {
namespace {

using attn::bf16x8_t;
using f32x4_t = __attribute__((ext_vector_type(4))) float;

constexpr int KBLK = 128;  // K per block: 4 MFMA steps of 32

__device__ __forceinline__ f32x4_t mfma16(bf16x8_t a, bf16x8_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8_t ld16(const unsigned short* p) {
  return *reinterpret_cast<const bf16x8_t*>(p);
}

template <int NT, int MT, int GB, int NW>
__global__ __launch_bounds__(NW * 64) void skinny_gemm_kernel(const unsigned short* __restrict__ x,
                                                              const unsigned short* __restrict__ w,
                                                              const unsigned short* __restrict__ bias,
                                                              unsigned short* __restrict__ y, int M, int N,
                                                              int K) {
  __shared__ f32x4_t red[NW][NT * MT][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16 * NT;
  const int nblk = K / KBLK;
  const int b0 = wave * nblk / NW, b1 = (wave + 1) * nblk / NW;
  const unsigned short* wrow[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) wrow[i] = w + (long)(n0 + 16 * i + r) * K + 32 * g;
  // token rows beyond M read row 0 (finite values) and are never stored
  const unsigned short* xrow[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    const int m = t * 16 + r;
    xrow[t] = x + (long)(m < M ? m : 0) * K + 32 * g;
  }
  f32x4_t acc[NT][MT];
#pragma unroll
  for (int i = 0; i < NT; ++i)
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[i][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  int b = b0;
  for (; b + GB <= b1; b += GB) {
    bf16x8_t a[GB][NT][4], xb[GB][MT][4];
#pragma unroll
    for (int u = 0; u < GB; ++u)
#pragma unroll
      for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int s = 0; s < 4; ++s) a[u][i][s] = ld16(wrow[i] + (long)(b + u) * KBLK + 8 * s);
#pragma unroll
    for (int u = 0; u < GB; ++u)
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int s = 0; s < 4; ++s) xb[u][t][s] = ld16(xrow[t] + (long)(b + u) * KBLK + 8 * s);
#pragma unroll
    for (int u = 0; u < GB; ++u)
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < NT; ++i)
#pragma unroll
          for (int t = 0; t < MT; ++t) acc[i][t] = mfma16(a[u][i][s], xb[u][t][s], acc[i][t]);
  }
  for (; b < b1; ++b) {
    bf16x8_t a[NT][4], xb[MT][4];
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int s = 0; s < 4; ++s) a[i][s] = ld16(wrow[i] + (long)b * KBLK + 8 * s);
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int s = 0; s < 4; ++s) xb[t][s] = ld16(xrow[t] + (long)b * KBLK + 8 * s);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int t = 0; t < MT; ++t) acc[i][t] = mfma16(a[i][s], xb[t][s], acc[i][t]);
  }
#pragma unroll
  for (int i = 0; i < NT; ++i)
#pragma unroll
    for (int t = 0; t < MT; ++t) red[wave][i * MT + t][lane] = acc[i][t];
  __syncthreads();
  // D layout: lane l holds D[row = 4(l/16) + i][col = l%16] = y[token col][weight row]
  for (int idx = threadIdx.x; idx < NT * MT * 64; idx += NW * 64) {
    const int it = idx >> 6, l = idx & 63;
    const int i = it / MT, t = it % MT;
    f32x4_t s = red[0][it][l];
#pragma unroll
    for (int v = 1; v < NW; ++v) s += red[v][it][l];
    const int m = t * 16 + (l & 15);
    if (m >= M) continue;
    const int n = n0 + 16 * i + 4 * (l >> 4);
    float o[4] = {s[0], s[1], s[2], s[3]};
    if (bias != nullptr) {
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] += bf2f(bias[n + j]);
    }
    ushort4 pk;
    pk.x = f2bf(o[0]);
    pk.y = f2bf(o[1]);
    pk.z = f2bf(o[2]);
    pk.w = f2bf(o[3]);
    *reinterpret_cast<ushort4*>(y + (long)m * N + n) = pk;
  }
}

// ---- x staged in LDS (v2, M <= 16) ---------------------------------------------------------------
// skinny_gemm_kernel gives every wave its own K range, so each wave also streams the 16 token
// rows of that range: at 16 tokens the token loads equal the weight loads (L2 traffic = the HBM
// stream; 2.5-2.9 TB/s vs 4.2-4.6 at one token).  Here a workgroup = 4 waves on 64 weight rows
// (one 16-row tile each, the 1-token streaming pattern: 64 B of a row per lane per K block, GB
// blocks in flight) and ONE K chunk of KC; the chunk's token rows are staged once in LDS (row
// stride KC*2 + 16 B: conflict-free ds_read_b128 across the 16 token rows) and shared by the 4
// waves, so token traffic is 1/4 of the weight stream.  K chunks = gridDim.y workgroups per row
// tile write fp32 partial tiles to ws [KS][M][N]; decode_finalize_kernel sums them (+ bias).
template <int GB>
__global__ __launch_bounds__(256) void decode_gemm_kernel(const unsigned short* __restrict__ x,
                                                          const unsigned short* __restrict__ w,
                                                          const unsigned short* __restrict__ bias,
                                                          unsigned short* __restrict__ y, float* __restrict__ ws,
                                                          int M, int N, int K, int KC) {
  extern __shared__ __attribute__((aligned(16))) unsigned char xs_raw[];
  unsigned short* xs = reinterpret_cast<unsigned short*>(xs_raw);
  const int XST = KC + 8;  // LDS row stride (elements)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 64 + wave * 16;
  const int kc0 = blockIdx.y * KC;
  const int kc = min(KC, K - kc0);  // this chunk's depth (multiple of 128)
  // token rows of the chunk -> LDS (rows >= M as zeros)
  const int c8 = kc >> 3;
  for (int i = threadIdx.x; i < 16 * c8; i += 256) {
    const int m = i / c8, c = i - m * c8;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (m < M) v = *reinterpret_cast<const uint4*>(x + (long)m * K + kc0 + c * 8);
    *reinterpret_cast<uint4*>(xs + m * XST + c * 8) = v;
  }
  __syncthreads();
  const unsigned short* wrow = w + (long)(n0 + r) * K + kc0 + 32 * g;
  const unsigned short* xrow = xs + r * XST + 32 * g;
  f32x4_t acc = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int nb = kc / KBLK;
  int b = 0;
  for (; b + GB <= nb; b += GB) {
    bf16x8_t a[GB][4];
#pragma unroll
    for (int u = 0; u < GB; ++u)
#pragma unroll
      for (int s = 0; s < 4; ++s) a[u][s] = ld16(wrow + (b + u) * KBLK + 8 * s);
    // every block of the batch in flight before the first MFMA (hipcc otherwise interleaves
    // loads and MFMAs to save registers: ~4 loads in flight, latency-bound)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < GB; ++u)
#pragma unroll
      for (int s = 0; s < 4; ++s)
        acc = mfma16(a[u][s], *reinterpret_cast<const bf16x8_t*>(xrow + (b + u) * KBLK + 8 * s), acc);
  }
  for (; b < nb; ++b) {
    bf16x8_t a[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) a[s] = ld16(wrow + b * KBLK + 8 * s);
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = mfma16(a[s], *reinterpret_cast<const bf16x8_t*>(xrow + b * KBLK + 8 * s), acc);
  }
  // D: lane holds [weight row n0 + 4g + i][token r]
  if (r >= M) return;
  const int n = n0 + 4 * g;
  if (ws == nullptr) {
    float o[4] = {acc[0], acc[1], acc[2], acc[3]};
    if (bias != nullptr) {
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] += bf2f(bias[n + j]);
    }
    ushort4 pk;
    pk.x = f2bf(o[0]);
    pk.y = f2bf(o[1]);
    pk.z = f2bf(o[2]);
    pk.w = f2bf(o[3]);
    *reinterpret_cast<ushort4*>(y + (long)r * N + n) = pk;
  } else {
    *reinterpret_cast<f32x4_t*>(ws + ((long)blockIdx.y * M + r) * N + n) = acc;
  }
}

// v3 (round 2): decode_gemm_kernel with the whole chunk's weight loads (NB <= 8 K blocks, 512 B per
// lane) issued BEFORE the token rows are staged, so the x-staging latency (L2 -> LDS, barrier)
// overlaps the first HBM round trip of the weight stream instead of preceding it; the block
// count is clamped on the load side (a short last chunk re-loads its last block, no per-load
// branch) and the MFMAs of past-the-end blocks are skipped (wave-uniform).
template <int NB>
__global__ __launch_bounds__(256) void decode_gemm_pre_kernel(const unsigned short* __restrict__ x,
                                                              const unsigned short* __restrict__ w,
                                                              const unsigned short* __restrict__ bias,
                                                              unsigned short* __restrict__ y, float* __restrict__ ws,
                                                              int M, int N, int K) {
  extern __shared__ __attribute__((aligned(16))) unsigned char xs_raw[];
  unsigned short* xs = reinterpret_cast<unsigned short*>(xs_raw);
  constexpr int KC = NB * KBLK, XST = KC + 8;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 64 + wave * 16;
  const int kc0 = blockIdx.y * KC;
  const int kc = min(KC, K - kc0);
  const int nb = kc / KBLK;
  // MFMA step s of lane group g reads k = 32 s + 8 g: a wave-instruction covers 64 contiguous bytes
  // of each of its 16 rows (k = 32 g + 8 s, 4 x 16 B at a 64-B stride per row, measured 0.6 % slower
  // in the decode step: profiles/decode_gemm_var_r5.txt)
  const int ko = 8 * g, ks = 32;
  const unsigned short* wrow = w + (long)(n0 + r) * K + kc0 + ko;
  bf16x8_t a[NB][4];
#pragma unroll
  for (int u = 0; u < NB; ++u) {
    const int bu = u < nb ? u : nb - 1;
#pragma unroll
    for (int s = 0; s < 4; ++s) a[u][s] = ld16(wrow + bu * KBLK + ks * s);
  }
  __builtin_amdgcn_sched_barrier(0);
  const int c8 = kc >> 3;
  for (int i = threadIdx.x; i < 16 * c8; i += 256) {
    const int m = i / c8, c = i - m * c8;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (m < M) v = *reinterpret_cast<const uint4*>(x + (long)m * K + kc0 + c * 8);
    *reinterpret_cast<uint4*>(xs + m * XST + c * 8) = v;
  }
  __syncthreads();
  const unsigned short* xrow = xs + r * XST + ko;
  f32x4_t acc = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < NB; ++u) {
    if (u < nb) {
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = mfma16(a[u][s], *reinterpret_cast<const bf16x8_t*>(xrow + u * KBLK + ks * s), acc);
    }
  }
  if (r >= M) return;
  const int n = n0 + 4 * g;
  if (ws == nullptr) {
    float o[4] = {acc[0], acc[1], acc[2], acc[3]};
    if (bias != nullptr) {
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] += bf2f(bias[n + j]);
    }
    ushort4 pk;
    pk.x = f2bf(o[0]);
    pk.y = f2bf(o[1]);
    pk.z = f2bf(o[2]);
    pk.w = f2bf(o[3]);
    *reinterpret_cast<ushort4*>(y + (long)r * N + n) = pk;
  } else {
    *reinterpret_cast<f32x4_t*>(ws + ((long)blockIdx.y * M + r) * N + n) = acc;
  }
}

// fp8 (OCP e4m3fn) weights, per-output-row fp32 scales (W8A16, decode only): the weight stream is
// half the bytes.  A lane's 16-B load holds 16 consecutive k of its row (k = 64 h + 16 g + [0, 16)
// in each 128-deep block, h = 0, 1), i.e. the A operands of two MFMA steps; e4m3 -> bf16 is exact
// (the f32 image's high half), and the B operand (token rows staged in LDS) follows the same k
// order.  The row scale multiplies the fp32 partial before it is stored, so the finalize passes
// (RoPE / SwiGLU / residual + RMSNorm) are the bf16 path's.
__device__ __forceinline__ bf16x8_t fp8x8_to_bf16x8(unsigned lo, unsigned hi) {
  float x[8];
  fp8x8_to_f32(make_uint2(lo, hi), x);
  bf16x8_t r;
  unsigned* w = reinterpret_cast<unsigned*>(&r);
#pragma unroll
  for (int j = 0; j < 4; ++j) w[j] = __builtin_amdgcn_perm(__float_as_uint(x[2 * j + 1]), __float_as_uint(x[2 * j]), 0x07060302u);
  return r;
}

template <int NB>
__global__ __launch_bounds__(256) void decode_gemm_w8_kernel(const unsigned short* __restrict__ x,
                                                             const unsigned char* __restrict__ w,
                                                             const float* __restrict__ wscale,
                                                             float* __restrict__ ws, int M, int N, int K) {
  extern __shared__ __attribute__((aligned(16))) unsigned char xs_raw[];
  unsigned short* xs = reinterpret_cast<unsigned short*>(xs_raw);
  constexpr int KC = NB * KBLK, XST = KC + 8;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 64 + wave * 16;
  const int kc0 = blockIdx.y * KC;
  const int kc = min(KC, K - kc0);
  const int nb = kc / KBLK;
  const unsigned char* wrow = w + (long)(n0 + r) * K + kc0 + 16 * g;
  uint4 a[NB][2];
#pragma unroll
  for (int u = 0; u < NB; ++u) {
    const int bu = u < nb ? u : nb - 1;
#pragma unroll
    for (int h = 0; h < 2; ++h) a[u][h] = *reinterpret_cast<const uint4*>(wrow + bu * KBLK + 64 * h);
  }
  __builtin_amdgcn_sched_barrier(0);
  const int c8 = kc >> 3;
  for (int i = threadIdx.x; i < 16 * c8; i += 256) {
    const int m = i / c8, c = i - m * c8;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (m < M) v = *reinterpret_cast<const uint4*>(x + (long)m * K + kc0 + c * 8);
    *reinterpret_cast<uint4*>(xs + m * XST + c * 8) = v;
  }
  __syncthreads();
  const unsigned short* xrow = xs + r * XST + 16 * g;
  f32x4_t acc = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < NB; ++u) {
    if (u < nb) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint4 q = a[u][h];
        acc = mfma16(fp8x8_to_bf16x8(q.x, q.y), *reinterpret_cast<const bf16x8_t*>(xrow + u * KBLK + 64 * h), acc);
        acc = mfma16(fp8x8_to_bf16x8(q.z, q.w), *reinterpret_cast<const bf16x8_t*>(xrow + u * KBLK + 64 * h + 8), acc);
      }
    }
  }
  if (r >= M) return;
  const int n = n0 + 4 * g;
  const float4 sc = *reinterpret_cast<const float4*>(wscale + n);
  acc[0] *= sc.x;
  acc[1] *= sc.y;
  acc[2] *= sc.z;
  acc[3] *= sc.w;
  *reinterpret_cast<f32x4_t*>(ws + ((long)blockIdx.y * M + r) * N + n) = acc;
}

// y[m][n] = bf16(sum_s ws[s][m][n] + bias[n]), 4 columns per thread
__global__ __launch_bounds__(256) void decode_finalize_kernel(const float* __restrict__ ws,
                                                              const unsigned short* __restrict__ bias,
                                                              unsigned short* __restrict__ y, int M, int N, int KS) {
  const long i = ((long)blockIdx.x * 256 + threadIdx.x) * 4;
  const long MN = (long)M * N;
  if (i >= MN) return;
  f32x4_t v = *reinterpret_cast<const f32x4_t*>(ws + i);
  for (int sidx = 1; sidx < KS; ++sidx) v += *reinterpret_cast<const f32x4_t*>(ws + sidx * MN + i);
  const int n = (int)(i % N);
  float o[4] = {v[0], v[1], v[2], v[3]};
  if (bias != nullptr) {
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] += bf2f(bias[n + j]);
  }
  ushort4 pk;
  pk.x = f2bf(o[0]);
  pk.y = f2bf(o[1]);
  pk.z = f2bf(o[2]);
  pk.w = f2bf(o[3]);
  *reinterpret_cast<ushort4*>(y + i) = pk;
}


// ---- fused decode epilogues (round 2): the finalize pass that sums the v2 K-chunk partials also
// runs the elementwise op that followed the projection, so a decode layer launches 3 fewer
// kernels and never round-trips the projection output through HBM.  Every epilogue first rounds
// the projection output to bf16 exactly as the unfused path stores it (sum + bias -> bf16), so
// the results match the unfused kernels (rope_fwd_kernel, swiglu_fwd_kernel: bit for bit;
// norm_fwd_kernel: up to the order of the sum of squares).
__device__ __forceinline__ f32x4_t sum_parts(const float* __restrict__ ws, long MN, int KS, long i) {
  f32x4_t v = *reinterpret_cast<const f32x4_t*>(ws + i);
  for (int s = 1; s < KS; ++s) v += *reinterpret_cast<const f32x4_t*>(ws + s * MN + i);
  return v;
}
// projection output element as the unfused GEMM stores it
__device__ __forceinline__ void round_out(const f32x4_t v, const unsigned short* __restrict__ bias, int n, float* o) {
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = bf2f(f2bf(v[j] + (bias != nullptr ? bf2f(bias[n + j]) : 0.f)));
}

// QKV projection -> RoPE (rotate-half) -> q out, K/V rows into the paged cache (slot < 0: skipped).
// thread = (token t, head h, 8-column slice c of each half of the head)
__global__ __launch_bounds__(256) void decode_fin_rope_kernel(const float* __restrict__ ws,
                                                              const unsigned short* __restrict__ bias,
                                                              const float* __restrict__ cosT,
                                                              const float* __restrict__ sinT,
                                                              const int* __restrict__ pos,
                                                              const int64_t* __restrict__ slots,
                                                              unsigned short* __restrict__ q,
                                                              void* __restrict__ kc, void* __restrict__ vc, int M,
                                                              int nq, int nkv, int D, int KS, bool kv8) {
  const int CH = D >> 4, NH = nq + 2 * nkv, half = D >> 1;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)M * NH * CH) return;
  const int c = idx % CH;
  const int h = (idx / CH) % NH;
  const int t = idx / ((long)CH * NH);
  const long N = (long)NH * D, MN = (long)M * N;
  const int na = h * D + c * 8, nb = na + half;
  float a[8], b[8], o1[8], o2[8];
  round_out(sum_parts(ws, MN, KS, t * N + na), bias, na, a);
  round_out(sum_parts(ws, MN, KS, t * N + na + 4), bias, na + 4, a + 4);
  round_out(sum_parts(ws, MN, KS, t * N + nb), bias, nb, b);
  round_out(sum_parts(ws, MN, KS, t * N + nb + 4), bias, nb + 4, b + 4);
  if (h < nq + nkv) {
    const long p = pos[t];
    const float4* cp = reinterpret_cast<const float4*>(cosT + p * half + c * 8);
    const float4* sp = reinterpret_cast<const float4*>(sinT + p * half + c * 8);
    float cs[8], sn[8];
    *reinterpret_cast<float4*>(cs) = cp[0];
    *reinterpret_cast<float4*>(cs + 4) = cp[1];
    *reinterpret_cast<float4*>(sn) = sp[0];
    *reinterpret_cast<float4*>(sn + 4) = sp[1];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o1[j] = a[j] * cs[j] - b[j] * sn[j];
      o2[j] = b[j] * cs[j] + a[j] * sn[j];
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o1[j] = a[j];
      o2[j] = b[j];
    }
  }
  if (h < nq) {
    unsigned short* dst = q + ((long)t * nq + h) * D;
    store8(dst + c * 8, o1);
    store8(dst + half + c * 8, o2);
  } else {
    const long sl = slots[t];
    if (sl < 0) return;
    const bool isk = h < nq + nkv;
    const long e = (sl * nkv + (isk ? h - nq : h - nq - nkv)) * (long)D;  // element index, either cache type
    cache_store8(isk ? kc : vc, e + c * 8, o1, kv8);
    cache_store8(isk ? kc : vc, e + half + c * 8, o2, kv8);
  }
}

// gate/up projection [M, 2F] -> act = silu(g) * u [M, F]; thread = 4 columns of one token
__global__ __launch_bounds__(256) void decode_fin_swiglu_kernel(const float* __restrict__ ws,
                                                                const unsigned short* __restrict__ bias,
                                                                unsigned short* __restrict__ act, int M, int F,
                                                                int KS) {
  const long i = ((long)blockIdx.x * 256 + threadIdx.x) * 4;  // index into act [M][F]
  if (i >= (long)M * F) return;
  const int m = i / F, n = i % F;
  const long N = 2L * F, MN = (long)M * N;
  float gv[4], uv[4];
  round_out(sum_parts(ws, MN, KS, m * N + n), bias, n, gv);
  round_out(sum_parts(ws, MN, KS, m * N + F + n), bias, F + n, uv);
  ushort4 pk;
  pk.x = f2bf(gv[0] * (1.f / (1.f + __expf(-gv[0]))) * uv[0]);
  pk.y = f2bf(gv[1] * (1.f / (1.f + __expf(-gv[1]))) * uv[1]);
  pk.z = f2bf(gv[2] * (1.f / (1.f + __expf(-gv[2]))) * uv[2]);
  pk.w = f2bf(gv[3] * (1.f / (1.f + __expf(-gv[3]))) * uv[3]);
  *reinterpret_cast<ushort4*>(act + i) = pk;
}

// row-parallel projection [M, N] + residual add + RMSNorm (the next sub-layer's input norm):
//   s = bf16(bf16(x W^T + b) + res) -> res_out,  y = bf16(s * rsqrt(mean(s^2) + eps) * w)
// workgroup = one token row of 1024 threads (4 columns each at N = 4096: all KS partial loads of a
// thread in flight at once; 256 threads ran latency-bound at ~12 us); the rounded row is kept in
// LDS between the two passes
__global__ __launch_bounds__(1024) void decode_fin_add_rmsnorm_kernel(const float* __restrict__ ws,
                                                                     const unsigned short* __restrict__ bias,
                                                                     const unsigned short* __restrict__ res,
                                                                     const unsigned short* __restrict__ nw,
                                                                     unsigned short* __restrict__ y,
                                                                     unsigned short* __restrict__ res_out, int M, int N,
                                                                     int KS, float eps) {
  extern __shared__ __attribute__((aligned(16))) float srow[];
  __shared__ float red[16];
  const int m = blockIdx.x;
  const long MN = (long)M * N, base = (long)m * N;
  float ss = 0.f;
  for (int n = threadIdx.x * 4; n < N; n += 4096) {
    float o[4];
    round_out(sum_parts(ws, MN, KS, base + n), bias, n, o);
    const ushort4 rv = *reinterpret_cast<const ushort4*>(res + base + n);
    const unsigned short r4[4] = {rv.x, rv.y, rv.z, rv.w};
    ushort4 pk;
    unsigned short* pp = reinterpret_cast<unsigned short*>(&pk);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pp[j] = f2bf(o[j] + bf2f(r4[j]));
      const float sv = bf2f(pp[j]);
      srow[n + j] = sv;
      ss += sv * sv;
    }
    *reinterpret_cast<ushort4*>(res_out + base + n) = pk;
  }
  const float rs = rsqrtf(block_sum<16>(ss, red) / (float)N + eps);  // (barrier: srow complete)
  for (int n = threadIdx.x * 4; n < N; n += 4096) {
    const ushort4 wv = *reinterpret_cast<const ushort4*>(nw + n);
    ushort4 pk;
    pk.x = f2bf(srow[n] * rs * bf2f(wv.x));
    pk.y = f2bf(srow[n + 1] * rs * bf2f(wv.y));
    pk.z = f2bf(srow[n + 2] * rs * bf2f(wv.z));
    pk.w = f2bf(srow[n + 3] * rs * bf2f(wv.w));
    *reinterpret_cast<ushort4*>(y + base + n) = pk;
  }
}

}  // namespace

// v3 (weight loads issued before the x staging) for the fused decode projections and config 25;
// knob decode_v3 = 0 keeps the v2 kernel there (A/B)
bool decode_v3() { return knob("decode_v3", 1) != 0; }

// v2 launch: KC = K chunk per workgroup (multiple of 128), GB = K blocks in flight per wave
template <int GB>
void launch_decode(const at::Tensor& x, const at::Tensor& w, const unsigned short* bp, at::Tensor& y, int M, int N,
                   int K, int KC) {
  LLMCTL_CHECK(M <= 16 && N % 64 == 0 && KC % KBLK == 0, "decode_gemm: M <= 16, N % 64 == 0");
  KC = std::min(KC, K);
  const int KS = (K + KC - 1) / KC;
  const size_t lds = (size_t)16 * (KC + 8) * 2;
  at::Tensor ws;
  float* wsp = nullptr;
  if (KS > 1) {
    ws = at::empty({(long)KS * M * N}, x.options().dtype(at::kFloat));
    wsp = ws.data_ptr<float>();
  }
  hipLaunchKernelGGL((decode_gemm_kernel<GB>), dim3(N / 64, KS), dim3(256), lds, stream(), bf_ptr(x), bf_ptr(w), bp,
                     bf_mut(y), wsp, M, N, K, KC);
  if (KS > 1) {
    const long n4 = (long)M * N / 4;
    hipLaunchKernelGGL(decode_finalize_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, stream(), wsp, bp,
                       bf_mut(y), M, N, KS);
  }
}

// v3 decode GEMM launch: K chunks of 1024 (KS = gridDim.y), 8 K blocks in flight per lane
void launch_pre(const unsigned short* x, const unsigned short* w, const unsigned short* bp, unsigned short* y,
                float* wsp, int M, int N, int K, int KS) {
  constexpr int KC = 1024;
  hipLaunchKernelGGL((decode_gemm_pre_kernel<KC / KBLK>), dim3(N / 64, KS), dim3(256), (size_t)16 * (KC + 8) * 2,
                     stream(), x, w, bp, y, wsp, M, N, K);
}

// v3 launch (KC = 1024): chunk partials + decode_finalize_kernel
void launch_decode_v3(const at::Tensor& x, const at::Tensor& w, const unsigned short* bp, at::Tensor& y, int M, int N,
                      int K) {
  LLMCTL_CHECK(M <= 16 && N % 64 == 0, "decode_gemm: M <= 16, N % 64 == 0");
  constexpr int KC = 1024;
  const int KS = (K + KC - 1) / KC;
  at::Tensor ws;
  float* wsp = nullptr;
  if (KS > 1) {
    ws = at::empty({(long)KS * M * N}, x.options().dtype(at::kFloat));
    wsp = ws.data_ptr<float>();
  }
  launch_pre(bf_ptr(x), bf_ptr(w), bp, bf_mut(y), wsp, M, N, K, KS);
  if (KS > 1) {
    const long n4 = (long)M * N / 4;
    hipLaunchKernelGGL(decode_finalize_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, stream(), wsp, bp,
                       bf_mut(y), M, N, KS);
  }
}

template <int NT, int MT, int GB, int NW>
void launch_skinny(const at::Tensor& x, const at::Tensor& w, const unsigned short* bp, at::Tensor& y, int M, int N,
                   int K) {
  LLMCTL_CHECK(N % (16 * NT) == 0, "skinny_linear: N must be a multiple of ", 16 * NT, " for this config");
  hipLaunchKernelGGL((skinny_gemm_kernel<NT, MT, GB, NW>), dim3(N / (16 * NT)), dim3(NW * 64), 0, stream(), bf_ptr(x),
                     bf_ptr(w), bp, bf_mut(y), M, N, K);
}

// config: 0 = automatic (measured best per shape, tools/skinny_sweep.py); 1-14: {NT, GB, NW} of
// skinny_gemm_kernel (MT follows M: 1 for M <= 16, else 2); 20-24: the LDS-staged v2 (M <= 16)
at::Tensor skinny_linear_cfg(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
                             int64_t config) {
  LLMCTL_CHECK(x.dim() == 2 && w.dim() == 2 && x.is_contiguous() && w.is_contiguous(), "skinny_linear: 2-D contiguous");
  LLMCTL_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16, "skinny_linear: bf16");
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  LLMCTL_CHECK(w.size(1) == K, "skinny_linear: K mismatch");
  LLMCTL_CHECK(M >= 1 && M <= 32 && N % 16 == 0 && K % KBLK == 0, "skinny_linear: needs M<=32, N%16==0, K%128==0");
  const unsigned short* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    LLMCTL_CHECK(bias->scalar_type() == at::kBFloat16 && bias->is_contiguous() && bias->numel() == N, "bias [N] bf16");
    bp = bf_ptr(*bias);
  }
  const c10::DeviceGuard guard(x.device());
  auto y = at::empty({M, N}, x.options());
  int c = (int)config;
  // automatic choice from tools/skinny_sweep.py (profiles/skinny_sweep_r2*.jsonl, uncached GPT-7B
  // weights): 4 waves x 8 K-blocks each in flight (c3) at <= 4 tokens and 17-32; at 5..16 tokens
  // the LDS-staged v2 (c23: QKV 3.78, up 3.89, down 3.16, LM head 4.2 TB/s at 16 tokens vs
  // hipBLASLt 3.55 / 3.35 / 2.07 / 4.16) except the 4096 x 4096 o-projection (2 waves x 8
  // blocks, c7)
  if (c == 0) {
    if (M > 4 && M <= 16) c = (N <= 4096 && K <= 4096) ? 7 : (N % 64 == 0 ? (decode_v3() ? 25 : 23) : 3);
    else c = 3;
  }
  const bool m1 = M <= 16;
  switch (c) {
    case 1: m1 ? launch_skinny<1, 1, 4, 8>(x, w, bp, y, M, N, K) : launch_skinny<1, 2, 2, 8>(x, w, bp, y, M, N, K); break;
    case 2: m1 ? launch_skinny<1, 1, 4, 4>(x, w, bp, y, M, N, K) : launch_skinny<1, 2, 2, 4>(x, w, bp, y, M, N, K); break;
    case 3: m1 ? launch_skinny<1, 1, 8, 4>(x, w, bp, y, M, N, K) : launch_skinny<1, 2, 4, 4>(x, w, bp, y, M, N, K); break;
    case 4: m1 ? launch_skinny<2, 1, 4, 4>(x, w, bp, y, M, N, K) : launch_skinny<2, 2, 2, 4>(x, w, bp, y, M, N, K); break;
    case 5: m1 ? launch_skinny<1, 1, 4, 2>(x, w, bp, y, M, N, K) : launch_skinny<1, 2, 2, 2>(x, w, bp, y, M, N, K); break;
    case 6: m1 ? launch_skinny<2, 1, 2, 8>(x, w, bp, y, M, N, K) : launch_skinny<2, 2, 1, 8>(x, w, bp, y, M, N, K); break;
    case 7: m1 ? launch_skinny<1, 1, 8, 2>(x, w, bp, y, M, N, K) : launch_skinny<1, 2, 4, 2>(x, w, bp, y, M, N, K); break;
    case 8: m1 ? launch_skinny<1, 1, 4, 1>(x, w, bp, y, M, N, K) : launch_skinny<1, 2, 2, 1>(x, w, bp, y, M, N, K); break;
    case 9: m1 ? launch_skinny<4, 1, 2, 4>(x, w, bp, y, M, N, K) : launch_skinny<4, 2, 1, 4>(x, w, bp, y, M, N, K); break;
    case 10: m1 ? launch_skinny<4, 1, 2, 8>(x, w, bp, y, M, N, K) : launch_skinny<4, 2, 1, 8>(x, w, bp, y, M, N, K); break;
    case 11: m1 ? launch_skinny<4, 1, 1, 8>(x, w, bp, y, M, N, K) : launch_skinny<4, 2, 1, 8>(x, w, bp, y, M, N, K); break;
    case 12: m1 ? launch_skinny<8, 1, 1, 8>(x, w, bp, y, M, N, K) : launch_skinny<8, 2, 1, 8>(x, w, bp, y, M, N, K); break;
    case 13: m1 ? launch_skinny<2, 1, 4, 8>(x, w, bp, y, M, N, K) : launch_skinny<2, 2, 2, 8>(x, w, bp, y, M, N, K); break;
    case 14: m1 ? launch_skinny<4, 1, 2, 2>(x, w, bp, y, M, N, K) : launch_skinny<4, 2, 1, 2>(x, w, bp, y, M, N, K); break;
    // v2 (token rows staged in LDS per K chunk, M <= 16): KC 1024 / 512 / 2048, 8 or 4 K blocks in flight
    case 20: launch_decode<8>(x, w, bp, y, M, N, K, 1024); break;
    case 21: launch_decode<4>(x, w, bp, y, M, N, K, 512); break;
    case 22: launch_decode<8>(x, w, bp, y, M, N, K, 2048); break;
    case 23: launch_decode<4>(x, w, bp, y, M, N, K, 1024); break;
    case 24: launch_decode<8>(x, w, bp, y, M, N, K, 4096); break;
    case 25: launch_decode_v3(x, w, bp, y, M, N, K); break;
    default: LLMCTL_CHECK(false, "skinny_linear: unknown config ", config);
  }
  return y;
}

at::Tensor skinny_linear(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias) {
  return skinny_linear_cfg(x, w, bias, 0);
}

// ---- fused decode projections (v2 GEMM partials + epilogue finalize), M <= 16 ------------------
namespace {
constexpr int kFusedKC = 1024;  // K chunk of the fused projections (config 23's)

void check_decode_operands(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
                           const char* who) {
  LLMCTL_CHECK(x.dim() == 2 && w.dim() == 2 && x.is_contiguous() && w.is_contiguous(), who, ": 2-D contiguous");
  LLMCTL_CHECK(x.is_cuda() && w.is_cuda() && x.scalar_type() == at::kBFloat16 &&
                   (w.scalar_type() == at::kBFloat16 || w.scalar_type() == at::kFloat8_e4m3fn),
               who, ": bf16 GPU activations, bf16 or fp8 (e4m3fn) weights");
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  LLMCTL_CHECK(w.size(1) == K && M >= 1 && M <= 16 && N % 64 == 0 && K % KBLK == 0, who,
               ": needs M <= 16, N % 64 == 0, K % 128 == 0 (got ", M, "x", N, "x", K, ")");
  if (bias.has_value() && bias->defined())
    LLMCTL_CHECK(bias->scalar_type() == at::kBFloat16 && bias->is_contiguous() && bias->numel() == N, who,
                 ": bias [N] bf16");
}

const unsigned short* bias_ptr(const c10::optional<at::Tensor>& bias) {
  return bias.has_value() && bias->defined() ? bf_ptr(*bias) : nullptr;
}

bool w_fp8(const at::Tensor& w) { return w.scalar_type() == at::kFloat8_e4m3fn; }

// x W^T as fp32 K-chunk partials ws [KS][M][N]; returns KS.  fp8 W: w_scale [N] fp32 row scales.
int decode_partials(const at::Tensor& x, const at::Tensor& w, at::Tensor& ws,
                    const c10::optional<at::Tensor>& w_scale = c10::nullopt) {
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  const int KC = std::min(kFusedKC, K);
  const int KS = (K + KC - 1) / KC;
  ws = at::empty({(long)KS * M * N}, x.options().dtype(at::kFloat));
  if (w_fp8(w)) {
    // (two 16-row tiles per wave, and K chunks of 512 / 2048, measured 3-6 % slower in the decode
    // step: profiles/decode_w8_r5.txt)
    LLMCTL_CHECK(w_scale.has_value() && w_scale->defined() && w_scale->scalar_type() == at::kFloat &&
                     w_scale->is_contiguous() && w_scale->numel() == N && w_scale->is_cuda(),
                 "fp8 decode weights need fp32 row scales [N] on the GPU");
    hipLaunchKernelGGL((decode_gemm_w8_kernel<kFusedKC / KBLK>), dim3(N / 64, KS), dim3(256),
                       (size_t)16 * (kFusedKC + 8) * 2, stream(), bf_ptr(x),
                       static_cast<const unsigned char*>(w.data_ptr()), w_scale->data_ptr<float>(),
                       ws.data_ptr<float>(), M, N, K);
  } else if (decode_v3())  // (its LDS row stride is the full chunk's, whatever K is)
    launch_pre(bf_ptr(x), bf_ptr(w), nullptr, nullptr, ws.data_ptr<float>(), M, N, K, KS);
  else
    hipLaunchKernelGGL((decode_gemm_kernel<4>), dim3(N / 64, KS), dim3(256), (size_t)16 * (KC + 8) * 2, stream(),
                       bf_ptr(x), bf_ptr(w), nullptr, nullptr, ws.data_ptr<float>(), M, N, K, KC);
  return KS;
}
}  // namespace

// x W^T as fp32 K-chunk partials [KS, M, N] (the fused decode attention sums them itself)
at::Tensor decode_linear_partials(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& w_scale) {
  check_decode_operands(x, w, c10::nullopt, "decode_linear_partials");
  const int M = x.size(0), N = w.size(0);
  const c10::DeviceGuard guard(x.device());
  at::Tensor ws;
  const int KS = decode_partials(x, w, ws, w_scale);
  return ws.view({KS, M, N});
}

// q [M, nq, D] = RoPE(x Wqkv^T + b)[:, :nq]; K/V rows RoPE'd / copied into the paged cache at slots
at::Tensor decode_qkv_rope_cache(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
                                 const at::Tensor& cosT, const at::Tensor& sinT, int64_t nq, int64_t nkv,
                                 const at::Tensor& positions, at::Tensor& k_cache, at::Tensor& v_cache,
                                 const at::Tensor& slots, const c10::optional<at::Tensor>& w_scale) {
  check_decode_operands(x, w, bias, "decode_qkv_rope_cache");
  const int M = x.size(0), N = w.size(0);
  const int NH = nq + 2 * nkv;
  LLMCTL_CHECK(N % NH == 0, "decode_qkv_rope_cache: qkv width not divisible by heads");
  const int D = N / NH;
  LLMCTL_CHECK(D % 16 == 0, "decode_qkv_rope_cache: head_dim must be a multiple of 16");
  LLMCTL_CHECK(cosT.is_cuda() && sinT.is_cuda() && cosT.scalar_type() == at::kFloat && sinT.scalar_type() == at::kFloat &&
                   cosT.is_contiguous() && sinT.is_contiguous() && cosT.dim() == 2 && cosT.size(1) == D / 2 &&
                   cosT.sizes() == sinT.sizes(),
               "decode_qkv_rope_cache: cos/sin must be contiguous fp32 [P, D/2] GPU tables");
  LLMCTL_CHECK(positions.scalar_type() == at::kInt && positions.is_contiguous() && positions.numel() == M,
               "decode_qkv_rope_cache: positions int32 [M]");
  LLMCTL_CHECK(slots.scalar_type() == at::kLong && slots.is_contiguous() && slots.numel() == M,
               "decode_qkv_rope_cache: slots int64 [M]");
  LLMCTL_CHECK(k_cache.is_contiguous() && v_cache.is_contiguous() && kv_cache_ok(k_cache) &&
                   v_cache.scalar_type() == k_cache.scalar_type() && v_cache.sizes() == k_cache.sizes() &&
                   k_cache.dim() == 4 && k_cache.size(2) == nkv && k_cache.size(3) == D,
               "decode_qkv_rope_cache: k/v cache contiguous bf16 or fp8 (e4m3fn) [blocks, block_size, Hkv, D]");
  const c10::DeviceGuard guard(x.device());
  at::Tensor ws;
  const int KS = decode_partials(x, w, ws, w_scale);
  auto q = at::empty({M, nq, D}, x.options());
  const long total = (long)M * NH * (D / 16);
  hipLaunchKernelGGL(decode_fin_rope_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream(),
                     ws.data_ptr<float>(), bias_ptr(bias), cosT.data_ptr<float>(), sinT.data_ptr<float>(),
                     positions.data_ptr<int>(), slots.data_ptr<int64_t>(), bf_mut(q), k_cache.data_ptr(),
                     v_cache.data_ptr(), M, (int)nq, (int)nkv, D, KS, kv_fp8(k_cache));
  return q;
}

// act [M, F] = silu(g) * u of the gate/up projection gu = x W^T + b  ([M, 2F], gate first)
at::Tensor decode_up_swiglu(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
                            const c10::optional<at::Tensor>& w_scale) {
  check_decode_operands(x, w, bias, "decode_up_swiglu");
  const int M = x.size(0), N = w.size(0), F = N / 2;
  const c10::DeviceGuard guard(x.device());
  at::Tensor ws;
  const int KS = decode_partials(x, w, ws, w_scale);
  auto act = at::empty({M, F}, x.options());
  const long n4 = (long)M * F / 4;
  hipLaunchKernelGGL(decode_fin_swiglu_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, stream(),
                     ws.data_ptr<float>(), bias_ptr(bias), bf_mut(act), M, F, KS);
  return act;
}

// (y, res_out): res_out = (x W^T + b) + res, y = rmsnorm(res_out) * norm_w
std::tuple<at::Tensor, at::Tensor> decode_linear_add_rmsnorm(const at::Tensor& x, const at::Tensor& w,
                                                             const c10::optional<at::Tensor>& bias,
                                                             const at::Tensor& res, const at::Tensor& norm_w,
                                                             double eps, const c10::optional<at::Tensor>& w_scale) {
  check_decode_operands(x, w, bias, "decode_linear_add_rmsnorm");
  const int M = x.size(0), N = w.size(0);
  LLMCTL_CHECK(res.is_contiguous() && res.scalar_type() == at::kBFloat16 && res.dim() == 2 && res.size(0) == M &&
                   res.size(1) == N,
               "decode_linear_add_rmsnorm: residual bf16 [M, N]");
  LLMCTL_CHECK(norm_w.is_contiguous() && norm_w.scalar_type() == at::kBFloat16 && norm_w.numel() == N,
               "decode_linear_add_rmsnorm: norm weight bf16 [N]");
  LLMCTL_CHECK(N <= 16384, "decode_linear_add_rmsnorm: N <= 16384 (row staged in LDS)");
  const c10::DeviceGuard guard(x.device());
  at::Tensor ws;
  const int KS = decode_partials(x, w, ws, w_scale);
  auto y = at::empty({M, N}, x.options());
  auto res_out = at::empty({M, N}, x.options());
  hipLaunchKernelGGL(decode_fin_add_rmsnorm_kernel, dim3(M), dim3(1024), (size_t)N * 4, stream(), ws.data_ptr<float>(),
                     bias_ptr(bias), bf_ptr(res), bf_ptr(norm_w), bf_mut(y), bf_mut(res_out), M, N, KS, (float)eps);
  return {y, res_out};
}

// y [M, N] = x W^T (+ b) with fp8 (e4m3fn) W and fp32 row scales: partials + decode_finalize_kernel
at::Tensor decode_linear_fp8(const at::Tensor& x, const at::Tensor& w, const at::Tensor& w_scale,
                             const c10::optional<at::Tensor>& bias) {
  check_decode_operands(x, w, bias, "decode_linear_fp8");
  LLMCTL_CHECK(w_fp8(w), "decode_linear_fp8: fp8 (e4m3fn) weights");
  const int M = x.size(0), N = w.size(0);
  const c10::DeviceGuard guard(x.device());
  at::Tensor ws;
  const int KS = decode_partials(x, w, ws, w_scale);
  auto y = at::empty({M, N}, x.options());
  const long n4 = (long)M * N / 4;
  hipLaunchKernelGGL(decode_finalize_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, stream(),
                     ws.data_ptr<float>(), bias_ptr(bias), bf_mut(y), M, N, KS);
  return y;
}

TORCH_LIBRARY_IMPL(llmctl, CUDA, m) {
  m.impl("decode_linear_fp8", &decode_linear_fp8);
  m.impl("skinny_linear", &skinny_linear);
  m.impl("skinny_linear_cfg", &skinny_linear_cfg);
  m.impl("decode_qkv_rope_cache", &decode_qkv_rope_cache);
  m.impl("decode_up_swiglu", &decode_up_swiglu);
  m.impl("decode_linear_partials", &decode_linear_partials);
  m.impl("decode_linear_add_rmsnorm", &decode_linear_add_rmsnorm);
}

}  // namespace llmctl
