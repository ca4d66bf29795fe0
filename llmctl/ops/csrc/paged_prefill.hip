// Prefill attention over the PAGED KV cache (chunked prefill / prefix reuse), gfx950, MFMA 32x32x16.
//
// Queries are the new tokens of N sequences packed back to back (no padding): sequence n owns
// rows [cu_q[n], cu_q[n+1]) of q / o and, after this step's cache write, ctx[n] cached tokens;
// its new tokens sit at positions ctx[n] - qlen .. ctx[n] - 1.  A query at position p attends
// keys 0..p, ALL read from the paged cache through the sequence's block table — the cached
// prefix (an earlier chunk, a prefix shared with another request, a sequence resumed after
// preemption) and the chunk itself are one key range.  Full prefill is the case ctx == qlen.
//
// Structure: the flash-attention forward (flash_attn_fwd.hip) with the K/V tile loads
// indirected through the block table —
//   * workgroup = 4 waves = 128 query rows of one (sequence, q-head); Q in registers;
//   * K/V tiles of 64 keys, global -> registers -> LDS (async-STAGE split); each 16-B piece's
//     row is looked up as cache[bt[n][key / bs] * bs + key % bs][hk][:];
//   * swapped S^T = K Q^T (key on registers, query on lane), exp2-domain online softmax with the
//     deferred (wave-uniform, 2^8 headroom) rescale, O^T += V^T P^T;
//   * the work list (sequence, 128-row q-block) is built on the host heaviest-first; q-heads of
//     one K/V head are adjacent in dispatch order (L2 reuse of the gathered K/V).
#include "attn_common.h"

namespace llmctl {
using namespace attn;
namespace {

constexpr int PQB = 128;  // query rows per workgroup
constexpr int PKB = 64;   // keys per tile
constexpr float kPRescaleTh = 8.f;

struct PPArgs {
  const unsigned short* q;
  const void* kc;  // bf16 or fp8 e4m3fn cache (FP8 template)
  const void* vc;
  unsigned short* o;
  const int* bt;    // [N, maxb] block tables
  const int* cu_q;  // [N + 1] packed query offsets
  const int* ctx;   // [N] cached tokens after this step (prefix + chunk)
  const int* work;  // [nwork] (sequence << 16) | q-block
  int Hq, Hkv, bs, maxb;
  long q_st, q_sh, o_st, o_sh;
  float scale_log2;
};

template <int HD, bool FP8 = false>
__global__ __launch_bounds__(256, 2) void paged_prefill_kernel(PPArgs a) {
  constexpr int NKS = HD / 16, NDB = HD / 32, ROWB = HD * 2, CPR = HD / 8;
  constexpr int LD_ITERS = PKB * CPR / 256;
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * PKB * ROWB];
  unsigned char* Ks = smem;
  unsigned char* Vs = smem + PKB * ROWB;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int hq = blockIdx.x % a.Hq;
  const int wk = a.work[blockIdx.x / a.Hq];
  const int n = wk >> 16, qblk = wk & 0xffff;
  const int hk = hq / (a.Hq / a.Hkv);
  const int q_begin = a.cu_q[n];
  const int qlen = a.cu_q[n + 1] - q_begin;
  const int ctx = a.ctx[n];
  const int pos0 = ctx - qlen;  // position of the chunk's first token
  const int q_row0 = qblk * PQB + wave * 32;
  const int my_q = q_row0 + r;
  const int my_pos = pos0 + my_q;
  const int* btn = a.bt + (long)n * a.maxb;
  const long kv_row = (long)a.Hkv * HD;  // elements between consecutive cache slots

  bf16x8_t qf[NKS];
  {
    const unsigned short* Qp = a.q + (long)(q_begin + min(my_q, qlen - 1)) * a.q_st + (long)hq * a.q_sh;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) qf[ks] = __builtin_bit_cast(bf16x8_t, gload16(Qp + ks * 16 + 8 * hh));
  }
  f32x16 o[NDB];
#pragma unroll
  for (int d = 0; d < NDB; ++d)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[d][i] = 0.f;
  float m_i = -INFINITY, l_i = 0.f;

  const int kv_end = min(ctx, pos0 + qblk * PQB + PQB);  // last visible key of the block + 1
  const int ntiles = (kv_end + PKB - 1) / PKB;

  uint4 kst[LD_ITERS], vst[LD_ITERS];
  auto issue = [&](int t) {
#pragma unroll
    for (int it = 0; it < LD_ITERS; ++it) {
      const int c = tid + 256 * it;
      const int row = c / CPR, ch = c % CPR;
      const int key = t * PKB + row;
      if (key < ctx) {
        const long slot = (long)btn[key / a.bs] * a.bs + key % a.bs;
        const long off = slot * kv_row + (long)hk * HD + ch * 8;
        kst[it] = cache_load8_bf16(a.kc, off, FP8);  // fp8: 8 B loaded, widened to the bf16 LDS image
        vst[it] = cache_load8_bf16(a.vc, off, FP8);
      } else {
        kst[it] = make_uint4(0, 0, 0, 0);
        vst[it] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int it = 0; it < LD_ITERS; ++it) {
      const int c = tid + 256 * it;
      const int row = c / CPR, ch = c % CPR;
      *reinterpret_cast<uint4*>(Ks + row_off<HD>(row, ch)) = kst[it];
      *reinterpret_cast<uint4*>(Vs + tr_off<HD>(row, ch)) = vst[it];
    }
  };

  if (ntiles > 0) issue(0);
  for (int t = 0; t < ntiles; ++t) {
    __syncthreads();
    commit();
    __syncthreads();
    if (t + 1 < ntiles) issue(t + 1);
    const int kv0 = t * PKB;
    if (kv0 > pos0 + q_row0 + 31) continue;  // tile entirely above this wave's diagonal

    f32x16 s[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int i = 0; i < 16; ++i) s[kb][i] = 0.f;
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const bf16x8_t kf = lds_read_b128(Ks, row_off<HD>(kb * 32 + r, 2 * ks + hh));
        s[kb] = mfma32(kf, qf[ks], s[kb]);
      }
    }
    const bool need_mask = (kv0 + PKB - 1 > pos0 + q_row0) || (kv0 + PKB > ctx);
    float mx = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float x = s[kb][i] * a.scale_log2;
        if (need_mask) {
          const int key = kv0 + kb * 32 + acc_row(i, hh);
          if (key > my_pos || key >= ctx) x = -INFINITY;
        }
        s[kb][i] = x;
        mx = fmaxf(mx, x);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    const bool grow = __builtin_amdgcn_ballot_w64(mx > m_i + kPRescaleTh) != 0;
    const float m_new = grow ? fmaxf(m_i, mx) : m_i;
    const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
    float rs = 0.f;
    bf16x8_t pb[2][2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      float p[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        p[i] = fast_exp2(s[kb][i] - m_use);
        rs += p[i];
      }
      pb[kb][0] = to_bf16x8(p);
      pb[kb][1] = to_bf16x8(p + 8);
    }
    rs += __shfl_xor(rs, 32);
    if (grow) {
      const float alpha = fast_exp2(m_i - m_use);
      l_i *= alpha;
#pragma unroll
      for (int d = 0; d < NDB; ++d)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[d][i] *= alpha;
    }
    l_i += rs;
    m_i = m_new;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int d = 0; d < NDB; ++d) {
          const bf16x8_t vf = tr_frag<HD>(Vs, kb * 32 + 16 * st, d * 32, lane);
          o[d] = mfma32(vf, pb[kb][st], o[d]);
        }
  }

  if (my_q < qlen) {
    const float inv = l_i > 0.f ? 1.f / l_i : 0.f;
    unsigned short* Op = a.o + (long)(q_begin + my_q) * a.o_st + (long)hq * a.o_sh;
#pragma unroll
    for (int d = 0; d < NDB; ++d)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int col = d * 32 + 8 * g + 4 * hh;
        unsigned short w4[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) w4[j] = f2bf(o[d][4 * g + j] * inv);
        *reinterpret_cast<uint2*>(Op + col) =
            make_uint2((unsigned)w4[0] | ((unsigned)w4[1] << 16), (unsigned)w4[2] | ((unsigned)w4[3] << 16));
      }
  }
}

}  // namespace

// q [T, Hq, D] packed new tokens; k_cache / v_cache [num_blocks, block_size, Hkv, D] (one layer);
// block_tables [N, maxb] int32; cu_q [N+1] int32; ctx_lens [N] int32; work [nwork] int32
// ((seq << 16) | q-block, heaviest first).  Returns o [T, Hq, D].
at::Tensor paged_prefill_attention(const at::Tensor& q, const at::Tensor& k_cache, const at::Tensor& v_cache,
                                   const at::Tensor& block_tables, const at::Tensor& cu_q, const at::Tensor& ctx_lens,
                                   const at::Tensor& work, double scale) {
  LLMCTL_CHECK(q.dim() == 3 && k_cache.dim() == 4 && v_cache.sizes() == k_cache.sizes(),
               "paged_prefill_attention: q [T,Hq,D], caches [blocks,bs,Hkv,D]");
  const int Hq = q.size(1), D = q.size(2), Hkv = k_cache.size(2), bs = k_cache.size(1);
  LLMCTL_CHECK(D == 64 || D == 128, "head_dim must be 64 or 128");
  LLMCTL_CHECK(k_cache.size(3) == D && Hq % Hkv == 0, "paged_prefill_attention: head shapes");
  LLMCTL_CHECK(q.scalar_type() == at::kBFloat16 && kv_cache_ok(k_cache) && v_cache.scalar_type() == k_cache.scalar_type(),
               "paged_prefill_attention: bf16 q, bf16 or fp8 (e4m3fn) caches");
  LLMCTL_CHECK(q.stride(2) == 1 && q.stride(0) % 8 == 0 && q.stride(1) % 8 == 0 &&
                   (reinterpret_cast<uintptr_t>(q.data_ptr()) & 15) == 0,
               "paged_prefill_attention: q rows 16-B aligned, d contiguous");
  LLMCTL_CHECK(k_cache.is_contiguous() && v_cache.is_contiguous(), "caches must be contiguous");
  for (const at::Tensor* t : {&block_tables, &cu_q, &ctx_lens, &work})
    LLMCTL_CHECK(t->is_cuda() && t->scalar_type() == at::kInt && t->is_contiguous(),
                 "paged_prefill_attention: int32 contiguous metadata on the GPU");
  const int N = ctx_lens.size(0);
  LLMCTL_CHECK(cu_q.numel() == N + 1 && block_tables.dim() == 2 && block_tables.size(0) == N,
               "paged_prefill_attention: metadata shapes");
  const c10::DeviceGuard g(q.device());
  auto o = at::empty_like(q, q.options().memory_format(at::MemoryFormat::Contiguous));
  const long nwork = work.numel();
  if (nwork == 0 || q.size(0) == 0) return o;
  PPArgs a{bf_ptr(q), k_cache.data_ptr(), v_cache.data_ptr(), bf_mut(o), block_tables.data_ptr<int>(), cu_q.data_ptr<int>(),
           ctx_lens.data_ptr<int>(), work.data_ptr<int>(), Hq, Hkv, bs, (int)block_tables.size(1),
           q.stride(0), q.stride(1), o.stride(0), o.stride(1), (float)(scale * 1.4426950408889634)};
  const dim3 grid((unsigned)(nwork * Hq)), block(256);
  const bool fp8 = kv_fp8(k_cache);
  if (D == 128 && fp8) hipLaunchKernelGGL((paged_prefill_kernel<128, true>), grid, block, 0, stream(), a);
  else if (D == 128) hipLaunchKernelGGL(paged_prefill_kernel<128>, grid, block, 0, stream(), a);
  else if (fp8) hipLaunchKernelGGL((paged_prefill_kernel<64, true>), grid, block, 0, stream(), a);
  else hipLaunchKernelGGL(paged_prefill_kernel<64>, grid, block, 0, stream(), a);
  return o;
}

TORCH_LIBRARY_IMPL(llmctl, CUDA, m) { m.impl("paged_prefill_attention", &paged_prefill_attention); }

}  // namespace llmctl
