// Flash-attention forward (causal / full, GQA) for gfx950 — MFMA 32x32x16 bf16.
//
// Structure (CDNA guide App. B "Fused attention prefill"):
//   * workgroup = 4 waves = 128 query rows of one (batch, q-head); each wave owns 32 rows;
//     two workgroups per CU (2 waves per SIMD: one wave's softmax VALU issues under the
//     other's MFMAs);
//   * Q fragments live in registers for the whole kernel (HD/16 x bf16x8 per lane);
//   * K/V tiles of 64 keys arrive by LDS-DMA (buffer_load_dwordx4 ... lds, source-swizzled)
//     into a 2-slot ring: one s_barrier per tile, the next tile's DMA is issued right after it
//     and lands under this tile's MFMAs.  The buffer resource is re-based per tile (SALU only)
//     and its record count stops at the last key, so keys past S read as zeros;
//   * "swapped" QK^T: S^T = K Q^T puts the key index in registers and the query on the
//     lane, so the online-softmax row max/sum are in-lane + one xor-32 shuffle, and P^T
//     is directly the B operand of O^T += V^T P^T (no P round-trip through LDS);
//   * K is read with ds_read_b128 from an XOR-swizzled row image (T2), V with
//     ds_read_b64_tr_b16 from a swizzled tr image (T10) — both bank-conflict free;
//   * exp2-domain softmax: the row max is taken on the raw scores and the 1/sqrt(d)*log2(e)
//     scale is folded into the exponent's FMA (p = 2^(s*c - m)), ~4 VALU per score;
//   * masking is a scalar-uniform choice per (wave, tile): only causal-diagonal / sequence-end /
//     document-boundary tiles run the masked softmax (branch-free selects), every other tile the
//     plain one — round 1's per-element divergent branches cost ~30 % of the loop's issue slots
//     (profiles/attn_fwd_isa_r2.txt);
//   * causal: tiles wholly above a wave's diagonal are skipped; dispatch is XCD-aware: each XCD
//     (workgroup i -> XCD i % 8) walks a contiguous range of heads with a head's q-blocks back
//     to back, heaviest first, so the few heads resident per XCD keep their K/V in its L2
//     (the head-major order kept ~48 heads = 48 MB of K/V live per 4 MB L2);
//   * packed sequences (optional ``doc_start[B,S]``: position where each token's document
//     begins, non-decreasing): key j is visible to query i iff doc_start[i] <= j <= i; the
//     K/V loop starts at the block's first document start, so the work is sum(doc_len^2);
//   * small grids (e.g. a single 2k-token prefill: 1 x 32 heads x 16 q-blocks = 512 workgroups,
//     all resident at once, so the run time is the heaviest block's): the K/V range of every
//     q-block is split over two workgroups that write bf16 partial outputs + fp32 LSEs, merged by a
//     combine kernel — halves the critical path of the causal tail.
// Outputs O [B,S,Hq,HD] bf16 and LSE [B,Hq,S] fp32 (natural log) for the backward pass.
#include <cstdlib>

#include "attn_common.h"

namespace llmctl {
using namespace attn;
namespace {

// workgroup shape (A/B knob FA_NW, see the host code): NW waves x 32 query rows, NBUF-slot ring
constexpr int KB = 64;   // keys per tile
constexpr float kRescaleTh = 8.f;  // log2-domain headroom of the deferred softmax rescale

struct FwdArgs {
  const unsigned short* q;
  const unsigned short* k;
  const unsigned short* v;
  unsigned short* o;
  float* lse;
  int B, S, Hq, Hkv;
  long q_sb, q_ss, q_sh;  // element strides (batch, seq, head); d is contiguous
  long k_sb, k_ss, k_sh;
  long v_sb, v_ss, v_sh;
  long o_sb, o_ss, o_sh;
  float scale_log2;  // softmax_scale * log2(e)
  const int* doc;    // [B, S] document start per token, or nullptr
  unsigned short* o_part;  // SPLIT: [2, B, S, Hq, HD] bf16 normalised partial outputs
  float* lse_part;   // SPLIT: [2, B, Hq, S] natural-log partial LSEs
  int prio;          // raise the wave priority over its MFMA phases (A/B knob fa_prio)
};

template <int HD, bool CAUSAL, bool DOC = false, bool SPLIT = false, int NW = 4, int NBUF = 2>
__global__ __launch_bounds__(NW * 64, 2) void fa_fwd_kernel(FwdArgs a) {
  constexpr int QB = NW * 32;  // query rows per workgroup
  constexpr int NTHR = NW * 64;
  constexpr int NKS = HD / 16;            // k-steps of QK^T
  constexpr int NDB = HD / 32;            // 32-wide d blocks of O
  constexpr int ROWB = HD * 2;            // bytes per LDS row
  constexpr int TILE = KB * ROWB;         // one K (or V) tile image
  constexpr int PPW = TILE / 1024 / NW;   // 1-KiB DMA pieces per wave per operand
  constexpr int SLOT = 2 * TILE;          // K | V
  static_assert(PPW * NW * 1024 == TILE, "pieces must split evenly over the waves");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[NBUF * SLOT];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const int nqb = (a.S + QB - 1) / QB;
  const int BH = a.B * a.Hq;
  int bh, rest;
  if (SPLIT || BH % 8) {
    bh = blockIdx.x % BH;
    rest = blockIdx.x / BH;
  } else {
    // XCD-aware order: workgroup i runs on XCD i % 8; XCD x walks the heads
    // [x*BH/8, (x+1)*BH/8) one after another, all q-blocks of a head back to back (heaviest
    // first), so the K/V stream of the ~4 heads resident on an XCD stays in its 4 MB L2
    const int x = blockIdx.x & 7, j = blockIdx.x >> 3;
    bh = x * (BH >> 3) + j / nqb;
    rest = j % nqb;
  }
  const int part = SPLIT ? rest & 1 : 0;
  const int qblk = nqb - 1 - (SPLIT ? rest >> 1 : rest);  // heaviest (largest causal span) first
  const int b = bh / a.Hq, hq = bh % a.Hq;
  const int hk = hq / (a.Hq / a.Hkv);
  const int q_row0 = qblk * QB + wave * 32;  // wave-uniform
  const int my_q = q_row0 + r;

  const unsigned short* Qp = a.q + b * a.q_sb + hq * a.q_sh;
  const unsigned short* Kp = a.k + b * a.k_sb + hk * a.k_sh;
  const unsigned short* Vp = a.v + b * a.v_sb + hk * a.v_sh;

  // zero the ring once: DMA of keys past S may leave LDS unwritten, and V rows must be finite
  // (P is exactly 0 there, but 0 * NaN is not)
#pragma unroll
  for (int i = 0; i < NBUF * SLOT / (NTHR * 16); ++i)
    *reinterpret_cast<uint4*>(smem + i * NTHR * 16 + tid * 16) = make_uint4(0, 0, 0, 0);

  // ---- Q fragments (B operand of S^T = K Q^T): Q[my_q][16ks + 8hh + j]
  bf16x8_t qf[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    uint4 u = make_uint4(0, 0, 0, 0);
    if (my_q < a.S) u = gload16(Qp + (long)my_q * a.q_ss + ks * 16 + 8 * hh);
    qf[ks] = __builtin_bit_cast(bf16x8_t, u);
  }

  f32x16 o[NDB];
#pragma unroll
  for (int d = 0; d < NDB; ++d)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[d][i] = 0.f;
  float m_i = -INFINITY, l_i = 0.f;  // running max (log2 domain, scaled) and row sum

  const int kv_end = CAUSAL ? min(a.S, qblk * QB + QB) : a.S;
  int ntiles = (kv_end + KB - 1) / KB;
  // packed documents: this lane's first visible key, the wave's min / max of it (doc_start is
  // non-decreasing) and the block's first tile
  int my_start = 0, w_min = 0, w_max = 0, t0 = 0;
  if constexpr (DOC) {
    const int* ds = a.doc + (long)b * a.S;
    my_start = ds[min(my_q, a.S - 1)];
    w_min = __builtin_amdgcn_readfirstlane(ds[min(q_row0, a.S - 1)]);
    w_max = __builtin_amdgcn_readfirstlane(ds[min(q_row0 + 31, a.S - 1)]);
    t0 = __builtin_amdgcn_readfirstlane(ds[min(qblk * QB, a.S - 1)]) / KB;
  }
  if constexpr (SPLIT) {  // part 0: tiles [t0, mid), part 1: [mid, ntiles) (holds the diagonal)
    const int mid = (t0 + ntiles) / 2;
    if (part == 0) ntiles = mid;
    else t0 = mid;
  }

  // ---- DMA: piece p = i*4 + wave of a tile image holds LDS bytes [p*1024, +1024), lane-linear;
  //      the source is permuted so the image is the swizzled one (K: row image, V: tr image)
  unsigned vk[PPW], vv[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int byte = (i * NW + wave) * 1024 + lane * 16;
    const int row = byte / ROWB, pch = (byte % ROWB) >> 4;
    vk[i] = (unsigned)((row * a.k_ss + ((pch ^ swz_row<HD>(row)) << 3)) * 2);
    vv[i] = (unsigned)((row * a.v_ss + ((pch ^ swz_tr<HD>(row)) << 3)) * 2);
  }
  const unsigned lds0 = lds_addr(smem);
  // tiles are issued in order; the next one's key row and K / V row pointers advance by one tile
  // per issue (no per-tile 64-bit products), its ring slot is a template constant
  int ik0 = t0 * KB;
  const unsigned short* kc = Kp + (long)ik0 * a.k_ss;
  const unsigned short* vc = Vp + (long)ik0 * a.v_ss;
  const long k_step = (long)KB * a.k_ss, v_step = (long)KB * a.v_ss;
  auto issue = [&](auto slot_c) __attribute__((always_inline)) {
    constexpr int SLC = decltype(slot_c)::value;
    const int nk = min(KB, a.S - ik0);
    i32x4_t rk = buf_rsrc(kc, (unsigned)(((nk - 1) * a.k_ss + HD) * 2));
    i32x4_t rv = buf_rsrc(vc, (unsigned)(((nk - 1) * a.v_ss + HD) * 2));
    // descriptor SGPRs may come from v_readfirstlane: VALU-written SGPR -> VMEM read needs 5
    // wait states, which hipcc does not pad into the asm below (guide §5.7 item 2)
    asm volatile("s_nop 4" : "+s"(rk), "+s"(rv));
    const unsigned slot = lds0 + (unsigned)(SLC * SLOT) + wave * 1024;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      buf_dma16(rk, vk[i], slot + i * NW * 1024);
      buf_dma16(rv, vv[i], slot + TILE + i * NW * 1024);
    }
    ik0 += KB;
    kc += k_step;
    vc += v_step;
  };

  const float c = a.scale_log2;
  const int key_hi = CAUSAL ? min(my_q, a.S - 1) : a.S - 1;  // last key this lane's row sees
  // V^T fragment offsets per 32-column d block (tr_frag_at): rows kb * 32 + 16 st are multiples of 16
  int vlo[NDB], vhi[NDB];
#pragma unroll
  for (int d = 0; d < NDB; ++d) tr_frag_offs<HD>(d * 32, lane, vlo[d], vhi[d]);
  // K row-fragment offsets per k-step: the row-image swizzle of rows kb * 32 + r depends on r only
  // (swz_row<HD>(kb * 32 + r) == swz_row<HD>(r)), so kb folds into the ds_read immediate
  int kofs[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) kofs[ks] = row_off<HD>(r, 2 * ks + hh);
  // retire the Q loads here: the first in-loop use would otherwise carry a compiler vmcnt(0)
  // on every iteration, i.e. wait for the just-issued DMA of the next tile
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) asm volatile("" ::"v"(qf[ks]));
  // one K/V tile: S^T = K Q^T, online softmax, O^T += V^T P^T.  MASK: per-score visibility
  auto tile = [&](bool need_mask, const unsigned char* Ks, const unsigned char* Vs, int kv0) __attribute__((always_inline)) {
    // MFMA phases run at raised wave priority: when both waves of a SIMD are ready, the one
    // feeding the matrix pipe issues first and the other's softmax VALU fills the gaps
    if (a.prio) __builtin_amdgcn_s_setprio(1);
    f32x16 s[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int i = 0; i < 16; ++i) s[kb][i] = 0.f;
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) s[kb] = mfma32(lds_read_b128(Ks, kb * 32 * (HD * 2) + kofs[ks]), qf[ks], s[kb]);
    }
    if (need_mask) {  // wave-uniform: a scalar branch around branch-free selects
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int key = kv0 + kb * 32 + acc_row(i, hh);
          bool ok = key <= key_hi;
          if constexpr (DOC) ok = ok && key >= my_start;
          s[kb][i] = ok ? s[kb][i] : -INFINITY;
        }
    }
    if (a.prio) __builtin_amdgcn_s_setprio(0);
    float mx = s[0][0];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int i = (kb == 0 ? 1 : 0); i < 16; ++i) mx = fmaxf(mx, s[kb][i]);
    mx = xor32_max(mx) * c;
    // deferred rescale: keep the running max while no row's max grew by more than kRescaleTh
    // (p = 2^(s - m) then stays <= 2^kRescaleTh, exact in fp32 and well inside bf16 range); the
    // decision is wave-uniform, and O, l and the LSE all use the same (possibly stale) m, so the
    // result is the exact softmax.  Skips the 16*NDB O multiplies and the alpha exp per tile.
    const bool grow = __builtin_amdgcn_ballot_w64(mx > m_i + kRescaleTh) != 0;
    const float m_new = grow ? fmaxf(m_i, mx) : m_i;
    const float nm = (m_new == -INFINITY) ? 0.f : -m_new;
    float rs = 0.f;
    bf16x8_t pb[2][2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      float p[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        p[i] = fast_exp2(__builtin_fmaf(s[kb][i], c, nm));
        rs += p[i];
      }
      pb[kb][0] = to_bf16x8(p);
      pb[kb][1] = to_bf16x8(p + 8);
    }
    rs = xor32_add(rs);
    if (grow) {
      const float alpha = fast_exp2(m_i + nm);
      l_i *= alpha;
#pragma unroll
      for (int d = 0; d < NDB; ++d)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[d][i] *= alpha;
    }
    l_i += rs;
    m_i = m_new;
    if (a.prio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int d = 0; d < NDB; ++d) o[d] = mfma32(tr_frag_at<HD>(Vs, kb * 32 + 16 * st, vlo[d], vhi[d]), pb[kb][st], o[d]);
    if (a.prio) __builtin_amdgcn_s_setprio(0);
  };

  __syncthreads();  // ring zeroed before any DMA lands in it
  // tile t lives in ring slot (t - t0) % NBUF, NBUF-1 tiles in flight; the slot is a template
  // constant (LDS offsets fold into the reads' immediates instead of costing address registers)
  auto step = [&](auto slot_c, int t) __attribute__((always_inline)) {
    constexpr int SL = decltype(slot_c)::value;
    // this wave's pieces of tile t landed (the younger tiles' 2*PPW-instruction groups may
    // still fly) ... and, after the barrier, every wave's; everyone is done with tile t-1
    if constexpr (NBUF == 3) {
      if (t + 1 < ntiles) vm_wait_n<2 * PPW>();
      else vm_wait_n<0>();
    } else {
      vm_wait_n<0>();
    }
    __builtin_amdgcn_s_barrier();
    if (t + NBUF - 1 < ntiles) issue(std::integral_constant<int, (SL + NBUF - 1) % NBUF>{});  // tile t-1's slot
    const int kv0 = t * KB;
    bool live = true;
    if constexpr (CAUSAL) live = kv0 <= q_row0 + 31;      // else: wholly above the wave's diagonal
    if constexpr (DOC) live = live && kv0 + KB > w_min;   // else: before every query's document
    if (live) {
      const bool need_mask = (CAUSAL && kv0 + KB - 1 > q_row0) || (kv0 + KB > a.S) || (DOC && kv0 < w_max);
      tile(need_mask, smem + SL * SLOT, smem + SL * SLOT + TILE, kv0);
    }
  };
  if (t0 < ntiles) issue(std::integral_constant<int, 0>{});
  if constexpr (NBUF == 3)
    if (t0 + 1 < ntiles) issue(std::integral_constant<int, 1>{});
  for (int t = t0; t < ntiles; t += NBUF) {
    step(std::integral_constant<int, 0>{}, t);
    if (t + 1 < ntiles) step(std::integral_constant<int, 1>{}, t + 1);
    if constexpr (NBUF == 3)
      if (t + 2 < ntiles) step(std::integral_constant<int, 2>{}, t + 2);
  }

  // ---- epilogue: O = O^T^T / l ; LSE (natural log)
  if constexpr (SPLIT) {
    if (my_q < a.S) {
      const float inv = l_i > 0.f ? 1.f / l_i : 0.f;
      // bf16 partials: each is a normalised output, rounded like the final one; the combine's
      // convex merge adds at most about half an ulp (fp32 partials: 69.9 vs 65.4 us per
      // single-prompt layer, tools/attn_prefill_split_ab.py)
      unsigned short* Op = a.o_part + ((((long)part * a.B + b) * a.S + my_q) * a.Hq + hq) * HD;
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
      if (hh == 0)
        a.lse_part[(((long)part * a.B + b) * a.Hq + hq) * a.S + my_q] =
            (l_i > 0.f) ? (m_i + __log2f(l_i)) * 0.69314718055994531f : -INFINITY;
    }
    return;
  }
  if (my_q < a.S) {
    const float inv = l_i > 0.f ? 1.f / l_i : 0.f;
    unsigned short* Op = a.o + b * a.o_sb + (long)my_q * a.o_ss + hq * a.o_sh;
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
    if (hh == 0) {
      const float lse = (l_i > 0.f) ? (m_i + __log2f(l_i)) * 0.69314718055994531f : -INFINITY;
      a.lse[((long)b * a.Hq + hq) * a.S + my_q] = lse;
    }
  }
}

// merge the two K/V-range halves: lse = logaddexp(l0, l1), o = o0 e^(l0-lse) + o1 e^(l1-lse)
template <int HD>
__global__ __launch_bounds__(256) void fa_combine_kernel(const unsigned short* __restrict__ o_part,
                                                         const float* __restrict__ lse_part,
                                                         unsigned short* __restrict__ o, float* __restrict__ lse,
                                                         int B, int S, int Hq, long o_sb, long o_ss, long o_sh) {
  constexpr int LPR = HD / 8;  // lanes per (b, s, h) row, 8 elements each
  const long gid = (long)blockIdx.x * 256 + threadIdx.x;
  const long row = gid / LPR;  // (b, s, h) in [B, S, Hq] order
  const int sub = gid % LPR;
  if (row >= (long)B * S * Hq) return;
  const int hq = row % Hq;
  const long bs = row / Hq;
  const int sq = bs % S;
  const int b = bs / S;
  const long li = ((long)b * Hq + hq) * S + sq;
  const long plane = (long)B * Hq * S;
  const float l0 = lse_part[li], l1 = lse_part[plane + li];
  const float m = fmaxf(l0, l1);
  float w0 = 0.f, w1 = 0.f, l = -INFINITY;
  if (m != -INFINITY) {
    const float e0 = __expf(l0 - m), e1 = __expf(l1 - m);
    l = m + __logf(e0 + e1);
    w0 = e0 / (e0 + e1);
    w1 = e1 / (e0 + e1);
  }
  const long ob = row * HD + sub * 8;
  const long osz = (long)B * S * Hq * HD;
  float out[8], x0[8], x1[8];
  load8(o_part + ob, x0);
  load8(o_part + osz + ob, x1);
#pragma unroll
  for (int j = 0; j < 8; ++j) out[j] = w0 * x0[j] + w1 * x1[j];
  store8(o + b * o_sb + (long)sq * o_ss + (long)hq * o_sh + sub * 8, out);
  if (sub == 0) lse[li] = l;
}

template <int NW, int NBUF>
std::tuple<at::Tensor, at::Tensor> fwd_launch(const at::Tensor& q, at::Tensor& o, at::Tensor& lse, FwdArgs& a, int B,
                                              int S, int Hq, int D, bool causal,
                                              const c10::optional<at::Tensor>& doc_start) {
  constexpr int QB = NW * 32, WG_PER_CU = NW == 4 ? 2 : 1;
  const int nqb = (S + QB - 1) / QB;
  dim3 grid((unsigned)(B * Hq * nqb)), block(NW * 64);
  auto s = stream();
  // a grid that the CUs hold in one residency round finishes when its heaviest causal block
  // does: split every block's K/V range over two workgroups
  bool split = causal && !(doc_start.has_value() && doc_start->defined()) && nqb >= 4 &&
               (long)B * Hq * nqb <= (long)WG_PER_CU * num_cus();
  // knob fa_split = 0 / 1 overrides the heuristic (-1: auto; autotuner knob, llmctl.plugins.autotuning)
  if (const int64_t e = knob("fa_split", -1); e == 0) split = false;
  else if (e == 1) split = causal && !(doc_start.has_value() && doc_start->defined()) && nqb >= 2;
  if (split) {
    auto o_part = at::empty({2, B, S, Hq, D}, q.options());
    auto lse_part = at::empty({2, B, Hq, S}, q.options().dtype(at::kFloat));
    a.o_part = bf_mut(o_part);
    a.lse_part = lse_part.data_ptr<float>();
    dim3 g2((unsigned)(2 * B * Hq * nqb));
    const long threads = (long)B * S * Hq * (D / 8);
    if (D == 128) {
      hipLaunchKernelGGL((fa_fwd_kernel<128, true, false, true, NW, NBUF>), g2, block, 0, s, a);
      hipLaunchKernelGGL(fa_combine_kernel<128>, dim3((threads + 255) / 256), dim3(256), 0, s, a.o_part, a.lse_part,
                         bf_mut(o), lse.data_ptr<float>(), B, S, Hq, o.stride(0), o.stride(1), o.stride(2));
    } else {
      hipLaunchKernelGGL((fa_fwd_kernel<64, true, false, true, NW, NBUF>), g2, block, 0, s, a);
      hipLaunchKernelGGL(fa_combine_kernel<64>, dim3((threads + 255) / 256), dim3(256), 0, s, a.o_part, a.lse_part,
                         bf_mut(o), lse.data_ptr<float>(), B, S, Hq, o.stride(0), o.stride(1), o.stride(2));
    }
    return {o, lse};
  }
  if (doc_start.has_value() && doc_start->defined()) {
    const at::Tensor& ds = *doc_start;
    LLMCTL_CHECK(causal, "flash_attn_fwd: doc_start (packed sequences) needs causal attention");
    LLMCTL_CHECK(ds.is_cuda() && ds.scalar_type() == at::kInt && ds.is_contiguous() && ds.dim() == 2 &&
                     ds.size(0) == B && ds.size(1) == S,
                 "flash_attn_fwd: doc_start must be contiguous int32 [B,S]");
    a.doc = ds.data_ptr<int>();
    if (D == 128) hipLaunchKernelGGL((fa_fwd_kernel<128, true, true, false, NW, NBUF>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((fa_fwd_kernel<64, true, true, false, NW, NBUF>), grid, block, 0, s, a);
    return {o, lse};
  }
  if (D == 128) {
    if (causal) hipLaunchKernelGGL((fa_fwd_kernel<128, true, false, false, NW, NBUF>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((fa_fwd_kernel<128, false, false, false, NW, NBUF>), grid, block, 0, s, a);
  } else {
    if (causal) hipLaunchKernelGGL((fa_fwd_kernel<64, true, false, false, NW, NBUF>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((fa_fwd_kernel<64, false, false, false, NW, NBUF>), grid, block, 0, s, a);
  }
  return {o, lse};
}

}  // namespace

std::tuple<at::Tensor, at::Tensor> flash_attn_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                                                  double scale, bool causal,
                                                  const c10::optional<at::Tensor>& doc_start) {
  LLMCTL_CHECK(q.is_cuda() && k.is_cuda() && v.is_cuda(), "flash_attn_fwd: GPU tensors");
  LLMCTL_CHECK(q.scalar_type() == at::kBFloat16 && k.scalar_type() == at::kBFloat16 &&
                   v.scalar_type() == at::kBFloat16,
               "flash_attn_fwd: bf16");
  LLMCTL_CHECK(q.dim() == 4 && k.dim() == 4 && v.dim() == 4, "q/k/v must be [B,S,H,D]");
  const int B = q.size(0), S = q.size(1), Hq = q.size(2), D = q.size(3);
  const int Hkv = k.size(2);
  LLMCTL_CHECK(k.size(0) == B && k.size(1) == S && v.sizes() == k.sizes() && k.size(3) == D,
               "k/v shape must be [B,S,Hkv,D] matching q");
  LLMCTL_CHECK(Hq % Hkv == 0, "Hq must be a multiple of Hkv");
  LLMCTL_CHECK(D == 64 || D == 128, "head_dim must be 64 or 128, got ", D);
  LLMCTL_CHECK(q.stride(3) == 1 && k.stride(3) == 1 && v.stride(3) == 1, "head_dim must be contiguous");
  for (const at::Tensor* t : {&q, &k, &v})
    LLMCTL_CHECK(t->stride(0) % 8 == 0 && t->stride(1) % 8 == 0 && t->stride(2) % 8 == 0 &&
                     (reinterpret_cast<uintptr_t>(t->data_ptr()) & 15) == 0,
                 "q/k/v strides must be multiples of 8 elements and 16-B aligned");
  const c10::DeviceGuard g(q.device());
  auto o = at::empty({B, S, Hq, D}, q.options());
  auto lse = at::empty({B, Hq, S}, q.options().dtype(at::kFloat));
  if (B * S * Hq == 0) return {o, lse};
  FwdArgs a{bf_ptr(q), bf_ptr(k), bf_ptr(v), bf_mut(o), lse.data_ptr<float>(), B, S, Hq, Hkv,
            q.stride(0), q.stride(1), q.stride(2), k.stride(0), k.stride(1), k.stride(2),
            v.stride(0), v.stride(1), v.stride(2), o.stride(0), o.stride(1), o.stride(2),
            (float)(scale * 1.4426950408889634), nullptr, nullptr, nullptr, 0};
  a.prio = knob("fa_prio", 1) != 0 ? 1 : 0;  // default on: 2-3 % at B12 S2048 (0: off, A/B)
  // workgroup shape: knob fa_nw = 8 -> 8 waves (256 rows) with a 3-slot ring, one workgroup per
  // CU; default 4 waves (128 rows) with a 2-slot ring, two per CU (A/B knob, tools/attn_bench.py)
  if (knob("fa_nw", 4) == 8) return fwd_launch<8, 3>(q, o, lse, a, B, S, Hq, D, causal, doc_start);
  return fwd_launch<4, 2>(q, o, lse, a, B, S, Hq, D, causal, doc_start);
}

TORCH_LIBRARY_IMPL(llmctl, CUDA, m) { m.impl("flash_attn_fwd", &flash_attn_fwd); }

}  // namespace llmctl
