// Paged KV cache: write kernel + decode attention over block tables (gfx950).
//
// KV layout: k_cache/v_cache [num_blocks, block_size, Hkv, D] bf16 — one token's K row is
// contiguous (D*2 bytes), a block holds block_size consecutive tokens of one sequence.
//
// Decode (one new token per sequence) is HBM-bound: every cached K/V byte is read once.
// Workgroup = one (sequence, kv-head, context split) = 4 waves; the `group = Hq/Hkv` query
// heads that share the kv head are handled together so GQA reads K/V once per group.  Inside a
// wave, 16 lanes cooperate on one token (8 contiguous bf16 of D=128 per lane: 16-B loads), so
// a wave-instruction covers 4 tokens; q·k is reduced over the 16 lanes with xor-shuffles.
// Each wave streams a contiguous slice of its split with an online softmax, U tokens per lane
// per iteration: all U block-table reads, then all 2U K/V loads are issued before the first
// use (with one token per iteration the loop is latency-bound: one 16-B load pair in flight
// per lane).  The 4 waves (and the 4 token groups within each wave) are merged through LDS.
// Small batches (N·Hkv workgroups, far fewer than the ~2k that cover 256 CUs' HBM latency)
// split the context over `nsplit` workgroups (flash-decoding): fp32 partials (O unnormalised,
// running max m in the log2 domain, sum l) + a combine kernel.  nsplit depends only on
// shapes (batch rounded up to the decode-graph bucket), so a captured hipGraph stays valid for
// any context lengths and graph / eager decode agree bit for bit.
#include <algorithm>
#include <cstdlib>

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

template <int D, int G, int U, bool FP8 = false>
__global__ __launch_bounds__(256) void paged_decode_kernel(const unsigned short* __restrict__ q,
                                                            const void* __restrict__ kc,
                                                            const void* __restrict__ vc,
                                                            const int* __restrict__ block_tables,
                                                            const int* __restrict__ ctx_lens,
                                                            unsigned short* __restrict__ out,
                                                            float* __restrict__ part_o, float* __restrict__ part_ml,
                                                            int Hq, int Hkv, int block_size, int max_blocks,
                                                            float scale_log2, int nsplit) {
  // EPL cache elements per lane per token: 8 (16 B of bf16), or 16 for fp8 caches with G <= 4 (the
  // same 16 B per load, so a wave-instruction covers twice the tokens: a half-width load per lane
  // would halve the bytes in flight of this latency-bound stream and gain nothing)
  constexpr int EPL = (FP8 && G <= 4) ? 16 : 8;
  constexpr int LPT = D / EPL;        // lanes per token (bf16: 16 for D=128, 8 for D=64)
  constexpr int TPW = 64 / LPT;       // tokens per wave-instruction
  __shared__ float sm_m[4 * TPW][G], sm_l[4 * TPW][G];
  __shared__ float sm_o[4 * TPW][G][D];
  const int seq = blockIdx.x / Hkv, hk = blockIdx.x % Hkv, split = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane % LPT;         // which EPL-element slice of D
  const int tg = lane / LPT;          // token group inside the wave
  const int L = ctx_lens[seq];
  const int* bt = block_tables + (long)seq * max_blocks;
  // q slices for the group's heads
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
  // this workgroup's context split, then a contiguous token slice per wave
  const int chunk = (L + nsplit - 1) / nsplit;
  const int c0 = min(L, split * chunk), c1 = min(L, c0 + chunk);
  const int per_wave = (c1 - c0 + 3) / 4;
  const int t0 = c0 + wave * per_wave, t1 = min(c1, t0 + per_wave);
  const long kv_row = (long)Hkv * D;
  for (int t = t0 + tg; t < t1; t += TPW * U) {
    int blk[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int tt = t + u * TPW;
      blk[u] = tt < t1 ? bt[tt / block_size] : -1;
    }
    float kf[U][EPL], vf[U][EPL];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int tt = t + u * TPW;
      if (blk[u] >= 0) {
        const long base = ((long)blk[u] * block_size + (tt % block_size)) * kv_row + (long)hk * D + sub * EPL;
        if constexpr (EPL == 16) {  // fp8: one 16-B load = 16 elements
          const uint4 ku = *reinterpret_cast<const uint4*>(static_cast<const unsigned char*>(kc) + base);
          const uint4 vu = *reinterpret_cast<const uint4*>(static_cast<const unsigned char*>(vc) + base);
          fp8x8_to_f32(make_uint2(ku.x, ku.y), kf[u]);
          fp8x8_to_f32(make_uint2(ku.z, ku.w), kf[u] + 8);
          fp8x8_to_f32(make_uint2(vu.x, vu.y), vf[u]);
          fp8x8_to_f32(make_uint2(vu.z, vu.w), vf[u] + 8);
        } else {
          cache_load8(kc, base, kf[u], FP8);
          cache_load8(vc, base, vf[u], FP8);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      // validity is uniform over the LPT lanes of a token group, so the shuffles below only
      // ever read lanes that take the same branch
      if (blk[u] < 0) continue;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < EPL; ++j) s += qv[g][j] * kf[u][j];
#pragma unroll
        for (int off = LPT / 2; off > 0; off >>= 1) s += __shfl_xor(s, off);
        s *= scale_log2;
        const float mn = fmaxf(m[g], s);
        const float a = exp2f(m[g] - mn), p = exp2f(s - mn);
        l[g] = l[g] * a + p;
#pragma unroll
        for (int j = 0; j < EPL; ++j) o[g][j] = o[g][j] * a + p * vf[u][j];
        m[g] = mn;
      }
    }
  }
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

// Context splits per (sequence, kv-head): enough workgroups for ~4-8 per CU, at least 128
// context slots per split, at most 16.  The batch is rounded up to a power of two, as the
// serving engine's decode-graph buckets are, so graph replay and eager decode pick the same
// split.  Knob decode_splits > 0 overrides (tests, A/B; llmctl.config.knobs).
int decode_splits(int N, int Hkv, int max_ctx) {
  if (const int64_t v = knob("decode_splits", 0); v > 0) return (int)std::min<int64_t>(v, 64);
  int np = 1;
  while (np < N) np *= 2;
  const int wgs = std::max(1, np * Hkv);
  // a (sequence, kv-head) grid of 512-1023 workgroups needs only ~4 per CU: GPT-7B, 16 x 2k decode
  // step 7.04 ms at 2 splits vs 7.11 at 4 (the auto value before), 7.5 at 3, 8.6 at 1
  // (profiles/serve_r2_session6.txt); other grids (unmeasured against this) keep ~8 per CU
  const int target = (wgs >= 512 && wgs < 1024) ? 1024 : 2048;
  return std::max(1, std::min({(target + wgs - 1) / wgs, max_ctx / 128, 16}));
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
#define LAUNCH(DD, GG, UU)                                                                                         \
  do {                                                                                                             \
    if (fp8)                                                                                                       \
      hipLaunchKernelGGL((paged_decode_kernel<DD, GG, UU, true>), grid, block, 0, s, q, k_cache.data_ptr(),        \
                         v_cache.data_ptr(), block_tables.data_ptr<int>(), context_lens.data_ptr<int>(),            \
                         bf_mut(out), po, pml, Hq, Hkv, bs, max_blocks, sl2, nsplit);                             \
    else                                                                                                           \
      hipLaunchKernelGGL((paged_decode_kernel<DD, GG, UU>), grid, block, 0, s, q, k_cache.data_ptr(),              \
                         v_cache.data_ptr(), block_tables.data_ptr<int>(), context_lens.data_ptr<int>(),            \
                         bf_mut(out), po, pml, Hq, Hkv, bs, max_blocks, sl2, nsplit);                             \
  } while (0)
  if (D == 128) {
    if (G == 1) LAUNCH(128, 1, 4);
    else if (G == 2) LAUNCH(128, 2, 4);
    else if (G == 4) LAUNCH(128, 4, 2);
    else if (G == 8) LAUNCH(128, 8, 2);
    else LLMCTL_CHECK(false, "GQA group must be 1/2/4/8");
  } else if (D == 64) {
    if (G == 1) LAUNCH(64, 1, 4);
    else if (G == 2) LAUNCH(64, 2, 4);
    else if (G == 4) LAUNCH(64, 4, 2);
    else if (G == 8) LAUNCH(64, 8, 2);
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
