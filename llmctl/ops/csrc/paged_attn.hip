// Paged KV cache: write kernel + decode attention over block tables (gfx950).
//
// KV layout: k_cache/v_cache [num_blocks, block_size, Hkv, D] bf16 — one token's K row is
// contiguous (D*2 bytes), a block holds block_size consecutive tokens of one sequence.
//
// Decode (one new token per sequence) is HBM-bound: every cached K/V byte is read once.
// Workgroup = one (sequence, kv-head, context split) = 4 waves; the `group = Hq/Hkv` query
// heads that share the kv head are handled together so GQA reads K/V once per group.  Inside a
// wave, LPT lanes cooperate on one token, each holding one 16-B slice of its K / V row (8 bf16,
// or 16 fp8 e4m3 elements), so a wave-instruction covers 64/LPT tokens; q.k is reduced over the
// LPT lanes with xor-shuffles.  Each wave streams a contiguous slice of its split, software-
// pipelined: stage i+1's raw K/V loads are in flight while stage i runs its online softmax
// (paged_decode_kernel below).  The 4 waves (and the token groups within each wave) are merged
// through LDS.  Small grids split the context over `nsplit` workgroups (flash-decoding): fp32
// partials (O unnormalised, running max m in the log2 domain, sum l) + a combine kernel.
// nsplit depends only on shapes (batch rounded up to the decode-graph bucket), so a captured
// hipGraph stays valid for any context lengths and graph / eager decode agree bit for bit.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace llmctl {
namespace {

__global__ __launch_bounds__(256) void kv_write_kernel(const unsigned short* __restrict__ k,
                                                        const unsigned short* __restrict__ v, void* __restrict__ kc,
                                                        void* __restrict__ vc, const int64_t* __restrict__ slots,
                                                        int N, int row8, bool fp8) {
  // row8 = Hkv*D/8 vectors per token; fp8 caches take 8 B per vector
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)N * row8) return;
  const int t = i / row8, c = i % row8;
  const long slot = slots[t];
  if (slot < 0) return;
  float x[8];
  load8(k + ((long)t * row8 + c) * 8, x);
  cache_store8(kc, (slot * row8 + c) * 8, x, fp8);
  load8(v + ((long)t * row8 + c) * 8, x);
  cache_store8(vc, (slot * row8 + c) * 8, x, fp8);
}

// Merge the 4 waves x TPW token groups' online-softmax partials (m, l in the log2 domain, O
// unnormalised) of one workgroup through LDS; write the normalised row (nsplit 1) or the split's
// fp32 partial for paged_combine_kernel.
template <int D, int G, int EPL>
__device__ __forceinline__ void decode_merge(const float (&m)[G], const float (&l)[G], const float (&o)[G][EPL],
                                             unsigned short* __restrict__ out, float* __restrict__ part_o,
                                             float* __restrict__ part_ml, int seq, int hk, int Hq, int split,
                                             int nsplit) {
  constexpr int LPT = D / EPL, TPW = 64 / LPT;
  __shared__ float sm_m[4 * TPW][G], sm_l[4 * TPW][G];
  __shared__ float sm_o[4 * TPW][G][D];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane % LPT, tg = lane / LPT;
  // publish per (wave, token-group) partials
  const int slot = wave * TPW + tg;
#pragma unroll
  for (int g = 0; g < G; ++g) {
    if (sub == 0) {
      sm_m[slot][g] = m[g];
      sm_l[slot][g] = l[g];
    }
#pragma unroll
    for (int j = 0; j < EPL; ++j) sm_o[slot][g][sub * EPL + j] = o[g][j];
  }
  __syncthreads();
  // combine 4*TPW partials: thread -> (g, d)
  for (int idx = threadIdx.x; idx < G * D; idx += 256) {
    const int g = idx / D, d = idx % D;
    float M = -INFINITY;
    for (int s = 0; s < 4 * TPW; ++s) M = fmaxf(M, sm_m[s][g]);
    float Ls = 0.f, O = 0.f;
    if (M != -INFINITY) {
      for (int s = 0; s < 4 * TPW; ++s) {
        const float w = exp2f(sm_m[s][g] - M);
        Ls += sm_l[s][g] * w;
        O += sm_o[s][g][d] * w;
      }
    }
    const long row = (long)seq * Hq + hk * G + g;
    if (nsplit == 1) {
      out[row * D + d] = f2bf(Ls > 0.f ? O / Ls : 0.f);
    } else {
      const long p = row * nsplit + split;
      part_o[p * D + d] = O;
      if (d == 0) {
        part_ml[2 * p] = M;
        part_ml[2 * p + 1] = Ls;
      }
    }
  }
}

// Software-pipelined form: the wave's token slice is walked in stages of U tokens per lane; the
// raw 16-B K/V loads of stage i+1 are issued before stage i is computed (two register buffers of
// raw cache bytes, converted at use), so a wave keeps its loads in flight through its own softmax
// work.  Every lane loads every stage (tokens past the slice re-read its last token and are
// masked to p = 0), keeping the control flow uniform and the vmcnt accounting exact.  Block ids
// come from a 64-block window held one per lane (ds_bpermute per token, a reload every 64
// blocks), so no block-table round trip precedes a K/V load.  The U tokens of a stage share one
// running-max update (one rescale of O per stage, not per token).
template <int D, int G, int U, bool FP8>
__global__ __launch_bounds__(256) void paged_decode_kernel(const unsigned short* __restrict__ q,
                                                             const void* __restrict__ kc,
                                                             const void* __restrict__ vc,
                                                             const int* __restrict__ block_tables,
                                                             const int* __restrict__ ctx_lens,
                                                             unsigned short* __restrict__ out,
                                                             float* __restrict__ part_o, float* __restrict__ part_ml,
                                                             int Hq, int Hkv, int block_size, int max_blocks,
                                                             float scale_log2, int nsplit) {
  constexpr int EPL = (FP8 && G <= 4) ? 16 : 8;  // elements per 16-B lane load (bf16 8, fp8 16)
  constexpr int EB = FP8 ? 1 : 2;                // bytes per element
  static_assert(EPL * EB == 16 || EPL * EB == 8, "slice of 8 or 16 B");
  constexpr int LPT = D / EPL, TPW = 64 / LPT, SPAN = TPW * U;
  using raw_t = typename std::conditional<EPL * EB == 16, uint4, uint2>::type;  // one lane's raw slice
  const int seq = blockIdx.x / Hkv, hk = blockIdx.x % Hkv, split = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane % LPT, tg = lane / LPT;
  const int L = ctx_lens[seq];
  const int* bt = block_tables + (long)seq * max_blocks;
  float qv[G][EPL];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int h = 0; h < EPL; h += 8) load8(q + ((long)seq * Hq + hk * G + g) * D + sub * EPL + h, qv[g] + h);
  float m[G], l[G], o[G][EPL];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m[g] = -INFINITY;
    l[g] = 0.f;
#pragma unroll
    for (int j = 0; j < EPL; ++j) o[g][j] = 0.f;
  }
  const int chunk = (L + nsplit - 1) / nsplit;
  const int c0 = min(L, split * chunk), c1 = min(L, c0 + chunk);
  const int per_wave = (c1 - c0 + 3) / 4;
  const int t0 = c0 + wave * per_wave, t1 = min(c1, t0 + per_wave);
  const int nst = t1 > t0 ? (t1 - t0 + SPAN - 1) / SPAN : 0;  // stages (wave-uniform)
  const long kv_row = (long)Hkv * D;
  const unsigned char* kb = static_cast<const unsigned char*>(kc);
  const unsigned char* vb = static_cast<const unsigned char*>(vc);
  int wbase = t0 / block_size;
  int wblk = bt[min(wbase + lane, max_blocks - 1)];
  auto issue = [&](int st, raw_t (&kr)[U], raw_t (&vr)[U]) {
    const int ts = t0 + st * SPAN;
    const int last = min(t1 - 1, ts + SPAN - 1) / block_size;
    if (last - wbase >= 64) {  // wave-uniform: slide the block-id window
      wbase = ts / block_size;
      wblk = bt[min(wbase + lane, max_blocks - 1)];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int tt = min(ts + tg + u * TPW, t1 - 1);
      const int b = __shfl(wblk, tt / block_size - wbase);
      const long e = ((long)b * block_size + (tt % block_size)) * kv_row + (long)hk * D + sub * EPL;
      kr[u] = *reinterpret_cast<const raw_t*>(kb + e * EB);
      vr[u] = *reinterpret_cast<const raw_t*>(vb + e * EB);
    }
  };
  auto unpack = [&](const raw_t& r, float* x) {
    if constexpr (FP8) {
      if constexpr (EPL == 16) {
        fp8x8_to_f32(make_uint2(r.x, r.y), x);
        fp8x8_to_f32(make_uint2(r.z, r.w), x + 8);
      } else {
        fp8x8_to_f32(r, x);
      }
    } else {
      const unsigned w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        x[2 * j] = __uint_as_float(w[j] << 16);
        x[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
      }
    }
  };
  auto compute = [&](int st, const raw_t (&kr)[U], const raw_t (&vr)[U]) {
    const int ts = t0 + st * SPAN;
    float sc[U][G];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float kf[EPL];
      unpack(kr[u], kf);
#pragma unroll
      for (int g = 0; g < G; ++g) {
        // four independent partial sums: a single serial FMA chain of EPL links sat on the
        // critical path of every stage (latency, not issue, bounds this loop)
        float a[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < EPL; ++j) a[j & 3] = fmaf(qv[g][j], kf[j], a[j & 3]);
        sc[u][g] = (a[0] + a[1]) + (a[2] + a[3]);
      }
    }
#pragma unroll
    for (int off = LPT / 2; off > 0; off >>= 1)
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int g = 0; g < G; ++g) sc[u][g] += __shfl_xor(sc[u][g], off);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool ok = ts + tg + u * TPW < t1;
#pragma unroll
      for (int g = 0; g < G; ++g) sc[u][g] = ok ? sc[u][g] * scale_log2 : -INFINITY;
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float mx = m[g];
#pragma unroll
      for (int u = 0; u < U; ++u) mx = fmaxf(mx, sc[u][g]);
      const float ms = mx == -INFINITY ? 0.f : mx;
      const float al = exp2f(m[g] - ms);
      l[g] *= al;
#pragma unroll
      for (int j = 0; j < EPL; ++j) o[g][j] *= al;
      m[g] = mx;
#pragma unroll
      for (int u = 0; u < U; ++u) sc[u][g] = exp2f(sc[u][g] - ms);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float vf[EPL];
      unpack(vr[u], vf);
#pragma unroll
      for (int g = 0; g < G; ++g) {
        l[g] += sc[u][g];
#pragma unroll
        for (int j = 0; j < EPL; ++j) o[g][j] += sc[u][g] * vf[j];
      }
    }
  };
  raw_t kA[U], vA[U], kB[U], vB[U];
  if (nst > 0) issue(0, kA, vA);
  for (int st = 0; st < nst; st += 2) {
    if (st + 1 < nst) issue(st + 1, kB, vB);
    compute(st, kA, vA);
    if (st + 1 >= nst) break;
    if (st + 2 < nst) issue(st + 2, kA, vA);
    compute(st + 1, kB, vB);
  }
  decode_merge<D, G, EPL>(m, l, o, out, part_o, part_ml, seq, hk, Hq, split, nsplit);
}

// out[row] = sum_s O_s 2^(m_s - M) / sum_s l_s 2^(m_s - M); empty splits carry m = -inf.
template <int D>
__global__ __launch_bounds__(D) void paged_combine_kernel(const float* __restrict__ part_o,
                                                          const float* __restrict__ part_ml,
                                                          unsigned short* __restrict__ out, int nsplit) {
  const long row = blockIdx.x;
  const int d = threadIdx.x;
  const float* ml = part_ml + row * nsplit * 2;
  float M = -INFINITY;
  for (int s = 0; s < nsplit; ++s) M = fmaxf(M, ml[2 * s]);
  float Ls = 0.f, O = 0.f;
  if (M != -INFINITY) {
    for (int s = 0; s < nsplit; ++s) {
      const float w = exp2f(ml[2 * s] - M);
      Ls += ml[2 * s + 1] * w;
      O += part_o[(row * nsplit + s) * D + d] * w;
    }
  }
  out[row * D + d] = f2bf(Ls > 0.f ? O / Ls : 0.f);
}

// Context splits per (sequence, kv-head): about 512 workgroups (2 per CU: each wave keeps two
// stages of loads in flight, so 8 waves per CU cover the HBM latency), at least 256 context slots
// per split, at most 64.  The batch is rounded up to a power of two, as the serving engine's
// decode-graph buckets are, so graph replay and eager decode pick the same split.  Measured
// (tools/paged_decode_bw.py, profiles/paged_decode_r5.txt): GPT-7B 16 x 2k best at 1 split
// (512 workgroups), 32 q / 8 kv heads 16 x 2k and 4 x 4k at 2-4, one 8k sequence at 16+.
// Knob decode_splits > 0 overrides (tests, A/B; llmctl.config.knobs).
int decode_splits(int N, int Hkv, int max_ctx) {
  if (const int64_t v = knob("decode_splits", 0); v > 0) return (int)std::min<int64_t>(v, 64);
  int np = 1;
  while (np < N) np *= 2;
  const int wgs = std::max(1, np * Hkv);
  return std::max(1, std::min({(512 + wgs - 1) / wgs, max_ctx / 256, 64}));
}

}  // namespace

void kv_cache_write(const at::Tensor& k, const at::Tensor& v, at::Tensor& k_cache, at::Tensor& v_cache,
                    const at::Tensor& slot_mapping) {
  LLMCTL_CHECK(k.is_contiguous() && v.is_contiguous() && k_cache.is_contiguous() && v_cache.is_contiguous(),
               "kv_cache_write: contiguous tensors");
  LLMCTL_CHECK(k.scalar_type() == at::kBFloat16 && kv_cache_ok(k_cache) && v_cache.scalar_type() == k_cache.scalar_type(),
               "kv_cache_write: bf16 K/V into bf16 or fp8 (e4m3fn) caches");
  LLMCTL_CHECK(slot_mapping.scalar_type() == at::kLong && slot_mapping.numel() == k.size(0),
               "slot_mapping: int64 [N]");
  const int N = k.size(0);
  const long row = k.numel() / std::max(N, 1);
  LLMCTL_CHECK(row % 8 == 0 && k_cache.size(2) * k_cache.size(3) == row, "kv row size mismatch");
  if (N == 0) return;
  const c10::DeviceGuard g(k.device());
  const int row8 = row / 8;
  const long total = (long)N * row8;
  hipLaunchKernelGGL(kv_write_kernel, dim3((total + 255) / 256), dim3(256), 0, stream(), bf_ptr(k), bf_ptr(v),
                     k_cache.data_ptr(), v_cache.data_ptr(), slot_mapping.data_ptr<int64_t>(), N, row8,
                     kv_fp8(k_cache));
}

namespace {
// launch the decode kernel (+ combine) for N sequences x Hq query heads
void launch_paged_decode(const unsigned short* q, const at::Tensor& k_cache,
                         const at::Tensor& v_cache, const at::Tensor& block_tables, const at::Tensor& context_lens,
                         at::Tensor& out, int N, int Hq, int D, double scale) {
  const int bs = k_cache.size(1), Hkv = k_cache.size(2);
  const int G = Hq / Hkv;
  const int max_blocks = block_tables.size(1);
  const float sl2 = (float)(scale * 1.4426950408889634);
  const int nsplit = decode_splits(N, Hkv, max_blocks * bs);
  at::Tensor part_o, part_ml;
  float *po = nullptr, *pml = nullptr;
  if (nsplit > 1) {
    part_o = at::empty({(long)N * Hq * nsplit * D}, out.options().dtype(at::kFloat));
    part_ml = at::empty({(long)N * Hq * nsplit * 2}, out.options().dtype(at::kFloat));
    po = part_o.data_ptr<float>();
    pml = part_ml.data_ptr<float>();
  }
  dim3 grid(N * Hkv, nsplit), block(256);
  auto s = stream();
  const bool fp8 = kv_fp8(k_cache);
#define LAUNCH(DD, GG)                                                                                             \
  do {                                                                                                             \
    if (fp8)                                                                                                       \
      hipLaunchKernelGGL((paged_decode_kernel<DD, GG, 2, true>), grid, block, 0, s, q, k_cache.data_ptr(),        \
                         v_cache.data_ptr(), block_tables.data_ptr<int>(), context_lens.data_ptr<int>(),            \
                         bf_mut(out), po, pml, Hq, Hkv, bs, max_blocks, sl2, nsplit);                             \
    else                                                                                                           \
      hipLaunchKernelGGL((paged_decode_kernel<DD, GG, (GG == 8 ? 4 : 2), false>), grid, block, 0, s, q,     \
                         k_cache.data_ptr(), v_cache.data_ptr(), block_tables.data_ptr<int>(),                     \
                         context_lens.data_ptr<int>(), bf_mut(out), po, pml, Hq, Hkv, bs, max_blocks, sl2, nsplit); \
  } while (0)
  if (D == 128) {
    if (G == 1) LAUNCH(128, 1);
    else if (G == 2) LAUNCH(128, 2);
    else if (G == 4) LAUNCH(128, 4);
    else if (G == 8) LAUNCH(128, 8);
    else LLMCTL_CHECK(false, "GQA group must be 1/2/4/8");
  } else if (D == 64) {
    if (G == 1) LAUNCH(64, 1);
    else if (G == 2) LAUNCH(64, 2);
    else if (G == 4) LAUNCH(64, 4);
    else if (G == 8) LAUNCH(64, 8);
    else LLMCTL_CHECK(false, "GQA group must be 1/2/4/8");
  } else {
    LLMCTL_CHECK(false, "head_dim must be 64 or 128");
  }
#undef LAUNCH
  if (nsplit > 1) {
    if (D == 128)
      hipLaunchKernelGGL(paged_combine_kernel<128>, dim3(N * Hq), dim3(128), 0, s, po, pml, bf_mut(out), nsplit);
    else
      hipLaunchKernelGGL(paged_combine_kernel<64>, dim3(N * Hq), dim3(64), 0, s, po, pml, bf_mut(out), nsplit);
  }
}

void check_paged_inputs(const at::Tensor& k_cache, const at::Tensor& v_cache, const at::Tensor& block_tables,
                        const at::Tensor& context_lens, int N, int Hq, int D) {
  LLMCTL_CHECK(k_cache.dim() == 4 && k_cache.is_contiguous() && v_cache.sizes() == k_cache.sizes() &&
                   v_cache.is_contiguous() && kv_cache_ok(k_cache) && v_cache.scalar_type() == k_cache.scalar_type(),
               "caches: contiguous bf16 or fp8 (e4m3fn) [blocks, block_size, Hkv, D]");
  LLMCTL_CHECK(block_tables.scalar_type() == at::kInt && block_tables.is_contiguous() &&
                   context_lens.scalar_type() == at::kInt && context_lens.is_contiguous(),
               "block_tables / context_lens must be contiguous int32");
  LLMCTL_CHECK(k_cache.size(3) == D && Hq % k_cache.size(2) == 0, "head shape mismatch");
  LLMCTL_CHECK(block_tables.dim() == 2 && block_tables.size(0) >= N && context_lens.numel() >= N,
               "block_tables [N, max_blocks] / context_lens [N]");
}
}  // namespace

at::Tensor paged_attention_decode(const at::Tensor& q, const at::Tensor& k_cache, const at::Tensor& v_cache,
                                  const at::Tensor& block_tables, const at::Tensor& context_lens, double scale) {
  LLMCTL_CHECK(q.dim() == 3 && q.is_contiguous() && q.scalar_type() == at::kBFloat16, "q: [N, Hq, D] bf16");
  const int N = q.size(0), Hq = q.size(1), D = q.size(2);
  check_paged_inputs(k_cache, v_cache, block_tables, context_lens, N, Hq, D);
  const c10::DeviceGuard g(q.device());
  auto out = at::empty_like(q);
  if (N == 0) return out;
  launch_paged_decode(bf_ptr(q), k_cache, v_cache, block_tables, context_lens, out, N, Hq, D, scale);
  return out;
}

TORCH_LIBRARY_IMPL(llmctl, CUDA, m) {
  m.impl("kv_cache_write", &kv_cache_write);
  m.impl("paged_attention_decode", &paged_attention_decode);
}

}  // namespace llmctl
