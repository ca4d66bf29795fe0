// Flash-attention backward (causal / full, GQA, packed documents) for gfx950 — MFMA 32x32x16 bf16.
//
// Recompute P from Q, K and the forward's LSE (CDNA guide App. B "Attention backward"):
//     S = Q K^T,  P = exp(scale S - lse),  dP = dO V^T,  dS = P (dP - delta),
//     dV = P^T dO,  dK = scale dS^T Q,  dQ = scale dS K          (delta = rowsum(dO * O))
//
// Two kernels, no atomics (the fused single-pass form summed dQ across key-block workgroups with
// fp32 atomics: 16 KB of atomic adds per 32x128 tile, ~3.4 GB per GPT-7B layer at mb 12, i.e. the
// ~1.3 TB/s chip-wide atomic rate alone was 2.6 ms of its 3.4 ms; MI355X_MICROARCH "Global float
// atomics").  Splitting costs 2 extra MFMA products (S and dP recomputed for dQ: 7 instead of 5)
// and buys: no dQ fp32 buffer memset / conversion pass, no dS LDS exchange, no atomics, and a
// shorter dependency chain in each kernel.
//
// fa_bwd_dkv_kernel — key-stationary: workgroup = 4 waves = 128 keys of one (batch, kv-head);
//   wave w owns keys [32w, 32w+32): their K / V fragments live in registers (B operands) and
//   dK^T / dV^T accumulate in registers across all query tiles of all q-heads of the GQA group.
//   Keys on the MFMA lane: the S / dP accumulators are directly the B operands of the dV^T and
//   dK^T products (accumulator-as-operand, guide §3).  Query tiles of 64 rows (two independent
//   32-row halves per wave: ILP between the MFMA chains and the exp/VALU work) stream through a
//   3-deep LDS ring filled by LDS-DMA (global_load_lds_dwordx4, source-swizzled "tr image" read
//   by ds_read_b128 rows AND ds_read_b64_tr_b16 columns, guide T10), one tile in flight across
//   each raw s_barrier behind a counted vmcnt; lse / delta (/ document starts) ride in the same
//   DMA ring as 256-B row-constant vectors.
// fa_bwd_dq_kernel — query-stationary, the forward's structure: workgroup = 4 waves = 128 query
//   rows of one (batch, q-head), Q and dO fragments in registers, K/V tiles of 64 keys arrive by
//   LDS-DMA into a 2-slot ring (one barrier per tile), XCD-aware block order, scalar-uniform
//   masking (only diagonal / sequence-end tiles run the selects); "swapped" products keep the
//   key on the registers so dS^T is directly the B operand of dQ^T += K^T dS^T.  dQ is written
//   once, in bf16.
// delta = rowsum(dO * O) is computed by the dQ kernel (its dO rows are in registers) and read by
// the dK/dV kernel launched after it.
#include "attn_common.h"

namespace llmctl {
using namespace attn;
namespace {

constexpr float LOG2E = 1.4426950408889634f;
constexpr int KV_KB = 128;  // keys per dK/dV workgroup
constexpr int KV_QT = 64;   // query rows per streamed tile
#ifndef LLMCTL_DKV_NBUF
#define LLMCTL_DKV_NBUF 2
#endif
// LDS ring depth of the dK/dV kernel (NB-1 Q/dO tiles in flight behind the one being computed;
// 33 KB per slot, one workgroup per CU either way: its registers allow one wave per SIMD).
// Measured at B12 S2048: 3 and 4 slots 1.5 % slower than 2 (2.015-2.021 vs 1.99 ms): its waits are
// LDS-read latency, not DMA (PMC: SQ_WAIT_ANY 21 % of wave cycles with either depth).
constexpr int KV_NBUF = LLMCTL_DKV_NBUF;
static_assert(KV_NBUF >= 2 && KV_NBUF <= 4, "dK/dV ring depth 2-4");
constexpr int DQ_QB = 128;  // query rows per dQ workgroup
constexpr int DQ_KB = 64;   // keys per dQ tile

struct BwdArgs {
  const unsigned short *q, *k, *v, *dout;
  const float* lse;    // [B,Hq,S] natural log
  const float* delta;  // [B,Hq,S]
  unsigned short *dq, *dk, *dv;  // [B,S,H,HD] contiguous
  int B, S, Hq, Hkv;
  long q_sb, q_ss, q_sh, k_sb, k_ss, k_sh, v_sb, v_ss, v_sh, do_sb, do_ss, do_sh;
  float scale, scale_log2;
  const int* doc;  // [B, S] document start per token (packed sequences), or nullptr
  // outputs: element strides per token (b*S + s) and per head of dq / dk / dv ([B,S,H,HD]
  // contiguous: H*HD and HD; straight into the QKV-projection gradient [T, (Hq+2Hkv)*HD]:
  // (Hq+2Hkv)*HD and HD with dk / dv offset to their head ranges)
  long dq_st, dk_st, dv_st;
  // RoPE backward fused into the stores (cos_t != nullptr): dq / dk rows rotated back by
  // position pos[token] (int32, or token % rope_S), table rows [pos][HD/2] fp32
  const float* cos_t;
  const float* sin_t;
  const int* rope_pos;
  int rope_S;
  // delta = rowsum(dO * O) computed by the dQ kernel (which holds the dO rows in registers) and
  // written to delta_w for the dK/dV kernel launched after it; o == nullptr: delta given
  const unsigned short* o;
  long o_sb, o_ss, o_sh;
  float* delta_w;
  // row constants of the dK/dV kernel, written by the dQ kernel launched before it:
  // rck_w[rc] = -lse / scale, rck_w[rc_n + rc] = -delta; the dK/dV kernel starts its S and dP
  // accumulators from them (S' = Q K^T - lse/scale, dP' = dO V^T - delta: p = exp2(c S'),
  // dS = p dP', no per-element subtract or LSE scaling)
  float* rck_w;
  long rc_n;
};

// dK^T / dV^T accumulation pinned to AGPRs: through the builtin, hipcc kept these 128 registers
// in VGPRs and shuttled the S / dP accumulators through AGPRs instead (~500 v_accvgpr moves per
// tile).  One asm statement issues a 16-row step's MFMAs for every d-block (dV^T += dO^T P^T and
// dK^T += Q^T dS^T interleaved), so hipcc can place nothing between them.  It pads no wait states
// into asm (guide §5.7 item 2), so the string carries them: s_nop 1 before (a just-written VALU
// operand, e.g. P^T / dS^T from v_cvt_pk) and s_nop 11 after (8-pass XDL result -> any non-MFMA
// reader or writer, e.g. a compiler v_accvgpr_mov of an accumulator).
template <int NDB>
__device__ __forceinline__ void dvdk_step(f32x16* dv, f32x16* dk, const bf16x8_t* da, const bf16x8_t* qa, bf16x8_t p,
                                          bf16x8_t ds) {
  if constexpr (NDB == 4) {
    asm volatile(
        "s_nop 1\n\t"
        "v_mfma_f32_32x32x16_bf16 %0, %8, %16, %0\n\t"
        "v_mfma_f32_32x32x16_bf16 %4, %12, %17, %4\n\t"
        "v_mfma_f32_32x32x16_bf16 %1, %9, %16, %1\n\t"
        "v_mfma_f32_32x32x16_bf16 %5, %13, %17, %5\n\t"
        "v_mfma_f32_32x32x16_bf16 %2, %10, %16, %2\n\t"
        "v_mfma_f32_32x32x16_bf16 %6, %14, %17, %6\n\t"
        "v_mfma_f32_32x32x16_bf16 %3, %11, %16, %3\n\t"
        "v_mfma_f32_32x32x16_bf16 %7, %15, %17, %7\n\t"
        "s_nop 11"
        : "+a"(dv[0]), "+a"(dv[1]), "+a"(dv[2]), "+a"(dv[3]), "+a"(dk[0]), "+a"(dk[1]), "+a"(dk[2]), "+a"(dk[3])
        : "v"(da[0]), "v"(da[1]), "v"(da[2]), "v"(da[3]), "v"(qa[0]), "v"(qa[1]), "v"(qa[2]), "v"(qa[3]), "v"(p),
          "v"(ds));
  } else {
    static_assert(NDB == 2, "head_dim 64 or 128");
    asm volatile(
        "s_nop 1\n\t"
        "v_mfma_f32_32x32x16_bf16 %0, %4, %8, %0\n\t"
        "v_mfma_f32_32x32x16_bf16 %2, %6, %9, %2\n\t"
        "v_mfma_f32_32x32x16_bf16 %1, %5, %8, %1\n\t"
        "v_mfma_f32_32x32x16_bf16 %3, %7, %9, %3\n\t"
        "s_nop 11"
        : "+a"(dv[0]), "+a"(dv[1]), "+a"(dk[0]), "+a"(dk[1])
        : "v"(da[0]), "v"(da[1]), "v"(qa[0]), "v"(qa[1]), "v"(p), "v"(ds));
  }
}

__device__ __forceinline__ void store_bf16x4(unsigned short* p, const float* x, float mul) {
  unsigned short w[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) w[j] = f2bf(x[j] * mul);
  *reinterpret_cast<uint2*>(p) =
      make_uint2((unsigned)w[0] | ((unsigned)w[1] << 16), (unsigned)w[2] | ((unsigned)w[3] << 16));
}

// Inverse rotate-half RoPE of one output row held as acc[d][4g + j] = x[32d + 8g + 4h + j] (HD =
// 128: d-blocks 0/1 pair with 2/3, i.e. column c with c + 64 in the same lane), then the bf16
// stores; rotation and softmax scale commute (both linear).
template <int HD, typename AccT>
__device__ __forceinline__ void store_row(unsigned short* dst, const AccT* acc, float mul, int hh,
                                          const float* cos_row, const float* sin_row) {
  constexpr int NDB = HD / 32;
  if (cos_row != nullptr) {
    constexpr int HB = NDB / 2;  // d-blocks per half
#pragma unroll
    for (int d = 0; d < HB; ++d)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = d * 32 + 8 * g + 4 * hh;  // < HD/2
        const float4 cs = *reinterpret_cast<const float4*>(cos_row + c);
        const float4 sn = *reinterpret_cast<const float4*>(sin_row + c);
        const float cv[4] = {cs.x, cs.y, cs.z, cs.w}, sv[4] = {sn.x, sn.y, sn.z, sn.w};
        float lo[4], hi[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float x1 = acc[d][4 * g + j], x2 = acc[d + HB][4 * g + j];
          lo[j] = x1 * cv[j] + x2 * sv[j];
          hi[j] = x2 * cv[j] - x1 * sv[j];
        }
        store_bf16x4(dst + c, lo, mul);
        store_bf16x4(dst + c + HD / 2, hi, mul);
      }
    return;
  }
#pragma unroll
  for (int d = 0; d < NDB; ++d)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float x[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) x[j] = acc[d][4 * g + j];
      store_bf16x4(dst + d * 32 + 8 * g + 4 * hh, x, mul);
    }
}

// =============================================================================================
// dK / dV
// =============================================================================================
template <int HD, bool CAUSAL, bool DOC>
__global__ __launch_bounds__(256, 1) void fa_bwd_dkv_kernel(BwdArgs a) {
  constexpr int NKS = HD / 16;
  constexpr int NDB = HD / 32;
  constexpr int ROWB = HD * 2;
  constexpr int TILE_B = KV_QT * ROWB;     // one Q (or dO) tile
  constexpr int NP = TILE_B / 1024 / 4;    // 1-KiB DMA pieces per wave per operand
  constexpr int RC_B = KV_QT * 4;          // one row-constant vector
  constexpr int BUF_B = 2 * TILE_B + 4 * RC_B;  // Q | dO | lse | delta | doc | (pad)
  constexpr int NB = KV_NBUF;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[NB * BUF_B];  // NB-slot ring

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const int nkb = (a.S + KV_KB - 1) / KV_KB;
  const int BH = a.B * a.Hkv;
  int bh, kblk;
  if (BH % 8) {
    bh = blockIdx.x % BH;
    kblk = blockIdx.x / BH;  // small kblk = most query tiles under causal: dispatched first
  } else {  // XCD-aware: XCD x walks kv-heads [x*BH/8, (x+1)*BH/8), a head's key blocks back to back
    const int x = blockIdx.x & 7, j = blockIdx.x >> 3;
    bh = x * (BH >> 3) + j / nkb;
    kblk = j % nkb;
  }
  const int b = bh / a.Hkv, hk = bh % a.Hkv;
  const int group = a.Hq / a.Hkv;
  const int k0 = kblk * KV_KB;
  const int wkey0 = k0 + wave * 32;  // wave-uniform
  const int my_key = wkey0 + r;

  // zero the ring (rows past S may stay unwritten by the DMA; every value read must be finite)
#pragma unroll
  for (int i = 0; i < NB * BUF_B / 4096; ++i)
    *reinterpret_cast<uint4*>(smem + i * 4096 + tid * 16) = make_uint4(0, 0, 0, 0);
  if (tid < (NB * BUF_B % 4096) / 16)
    *reinterpret_cast<uint4*>(smem + (NB * BUF_B / 4096) * 4096 + tid * 16) = make_uint4(0, 0, 0, 0);
  __syncthreads();

  const unsigned lds0 = lds_addr(smem);
  // ---- this wave's K / V fragments (B operands): lane holds X[my_key][16ks + 8hh + j]
  bf16x8_t kf[NKS], vf[NKS];
  {
    const int kc = min(my_key, a.S - 1);  // keys past S: real finite data, P masked to 0
    const unsigned short* Kp = a.k + b * a.k_sb + hk * a.k_sh + (long)kc * a.k_ss + 8 * hh;
    const unsigned short* Vp = a.v + b * a.v_sb + hk * a.v_sh + (long)kc * a.v_ss + 8 * hh;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      kf[ks] = __builtin_bit_cast(bf16x8_t, gload16(Kp + 16 * ks));
      vf[ks] = __builtin_bit_cast(bf16x8_t, gload16(Vp + 16 * ks));
    }
    // retire these loads HERE: a compiler wait inside the tile loop would be a vmcnt(0) that also
    // drains the (compiler-invisible) LDS-DMA prefetch of the next tile
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) asm volatile("" ::"v"(kf[ks]), "v"(vf[ks]));
  }

  f32x16 dk[NDB], dv[NDB];
#pragma unroll
  for (int d = 0; d < NDB; ++d)
#pragma unroll
    for (int i = 0; i < 16; ++i) dk[d][i] = dv[d][i] = 0.f;

  const int q_start = CAUSAL ? k0 : 0;  // k0 is a multiple of KV_QT
  int q_end = a.S;
  if constexpr (DOC) {
    // queries whose document starts after this block's last key see none of its keys
    const int* ds = a.doc + (long)b * a.S;
    int lo = min(k0 + KV_KB, a.S), hi = a.S;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (ds[mid] > k0 + KV_KB - 1) hi = mid;
      else lo = mid + 1;
    }
    q_end = __builtin_amdgcn_readfirstlane(lo);
  }
  const int nq = q_end > q_start ? (q_end - q_start + KV_QT - 1) / KV_QT : 0;
  const int ntiles = group * nq;
  // ---- DMA of tile (g, qi) into ring slot t % NB: every wave issues exactly 2*NP+1 instructions;
  //      buffer descriptors re-based per tile (SALU), per-lane offsets fixed: the tr image is
  //      built by permuting the source rows/chunks; rows past S read as zeros
  unsigned vq[NP], vd[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int byte = (i * 4 + wave) * 1024 + lane * 16;
    const int row = byte / ROWB;
    const int lch = ((byte % ROWB) >> 4) ^ swz_tr<HD>(row);
    vq[i] = (unsigned)((row * a.q_ss + lch * 8) * 2);
    vd[i] = (unsigned)((row * a.do_ss + lch * 8) * 2);
  }
  // wave 0: -lse/scale, 1: -delta (rck_w, from the dQ kernel), 2: doc (DOC), 3: pad.  The row
  // constants land in accumulator-register order: LDS word 32h + 16hh + 4gq + j holds row
  // 32h + 8gq + 4hh + j (the row of register 4gq+j of lane half hh in half-tile h)
  const float* rc_src = a.rck_w + (wave == 1 ? a.rc_n : 0);
  const unsigned rc_off =
      (DOC && wave == 2) ? lane * 4
                         : (unsigned)((32 * (lane >> 5) + 8 * ((lane >> 2) & 3) + 4 * ((lane >> 4) & 1) + (lane & 3)) * 4);
  // scalar state of the tile being issued, advanced incrementally (a 64-row step, or the next
  // q-head of the group at the end of the block's query range): no per-tile 64-bit products
  int iq0 = q_start;  // its first row
  const unsigned short* qh = a.q + b * a.q_sb + (long)(hk * group) * a.q_sh;  // head rows 0
  const unsigned short* dh = a.dout + b * a.do_sb + (long)(hk * group) * a.do_sh;
  const float* rh = rc_src + ((long)b * a.Hq + hk * group) * a.S;
  const unsigned short* qc = qh + (long)q_start * a.q_ss;  // its first row in each operand
  const unsigned short* dc = dh + (long)q_start * a.do_ss;
  const long q_step = (long)KV_QT * a.q_ss, d_step = (long)KV_QT * a.do_ss;
  constexpr int PT = 2 * NP + 1;  // DMA instructions per wave per tile
  auto issue = [&](auto slot_c) __attribute__((always_inline)) {
    constexpr int SLC = decltype(slot_c)::value;
    const int nr = min(KV_QT, a.S - iq0);
    i32x4_t rq = buf_rsrc(qc, (unsigned)(((nr - 1) * a.q_ss + HD) * 2));
    i32x4_t rd = buf_rsrc(dc, (unsigned)(((nr - 1) * a.do_ss + HD) * 2));
    i32x4_t rr = (DOC && wave == 2) ? buf_rsrc(a.doc + (long)b * a.S + iq0, (unsigned)(nr * 4))
                                    : buf_rsrc(rh + iq0, (unsigned)(nr * 4));
    // descriptor SGPRs may come from v_readfirstlane: 5 wait states before a VMEM reads them
    asm volatile("s_nop 4" : "+s"(rq), "+s"(rd), "+s"(rr));
    const unsigned slot = lds0 + (unsigned)(SLC * BUF_B);
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      buf_dma16(rq, vq[i], slot + (i * 4 + wave) * 1024);
      buf_dma16(rd, vd[i], slot + TILE_B + (i * 4 + wave) * 1024);
    }
    buf_dma4(rr, rc_off, slot + 2 * TILE_B + wave * RC_B);
    iq0 += KV_QT;
    qc += q_step;
    dc += d_step;
    if (iq0 >= q_end) {  // next q-head of the group
      iq0 = q_start;
      qh += a.q_sh;
      dh += a.do_sh;
      rh += a.S;
      qc = qh + (long)q_start * a.q_ss;
      dc = dh + (long)q_start * a.do_ss;
    }
  };

  if (ntiles > 0) issue(std::integral_constant<int, 0>{});
  if constexpr (NB >= 3)
    if (ntiles > 1) issue(std::integral_constant<int, 1>{});
  if constexpr (NB >= 4)
    if (ntiles > 2) issue(std::integral_constant<int, 2>{});
  int qi = 0;  // q-tile index of tile t
  auto step = [&](auto slot_c, int t) __attribute__((always_inline)) {
    constexpr int SL = decltype(slot_c)::value;
    // this wave's DMA of tile t landed (those of the younger tiles in flight may not have) ...
    const int younger = min(NB - 2, ntiles - 1 - t);
    if (NB >= 4 && younger >= 2) vm_wait_n<(NB >= 4 ? 2 * PT : 0)>();
    else if (NB >= 3 && younger >= 1) vm_wait_n<(NB >= 3 ? PT : 0)>();
    else vm_wait_n<0>();
    __builtin_amdgcn_s_barrier();       // ... and every other wave's; everyone is done with t-1
    // tile t+NB-1 goes into tile t-1's slot
    if (t + NB - 1 < ntiles) issue(std::integral_constant<int, (SL + NB - 1) % NB>{});
    const int q0 = q_start + qi * KV_QT;
    if (++qi == nq) qi = 0;
    // wave-uniform tile classes: all of this wave's keys after all of the tile's rows -> nothing
    // to do; diagonal / sequence-end / document tiles -> masked softmax; the rest -> plain
    if (CAUSAL && wkey0 > q0 + KV_QT - 1) return;
    const bool need_mask = DOC || (CAUSAL && wkey0 + 31 > q0) || (q0 + KV_QT > a.S) || (wkey0 + 31 >= a.S);
    const unsigned char* Qs = smem + SL * BUF_B;
    const unsigned char* Ds = Qs + TILE_B;
    const float* lse_s = reinterpret_cast<const float*>(Ds + TILE_B);
    const float* del_s = lse_s + KV_QT;
    const int* doc_s = reinterpret_cast<const int*>(del_s + KV_QT);

    // ---- per 32-row half h: S = Q K^T, dP = dO V^T (q on regs, key on lane), then
    //      dV^T += dO^T P and dK^T += Q^T dS (sum over the half's rows = the registers).
    //      One wave per SIMD: nothing else hides LDS latency, so each phase's fragments are read
    //      as a batch ahead of its MFMAs (the transposed ones before the softmax VALU).
    //      (Interleaving half 1's S/dP MFMAs with half 0's softmax through sched_group_barrier
    //      measured 2 % slower: 1.31 vs 1.28 ms at B12 S2048.)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      f32x16 s, dp;
      {
        bf16x8_t qa[NKS], da[NKS];
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          qa[ks] = lds_read_b128(Qs, tr_off<HD>(32 * h + r, 2 * ks + hh));
          da[ks] = lds_read_b128(Ds, tr_off<HD>(32 * h + r, 2 * ks + hh));
        }
        // accumulators start at the row constants -lse/scale and -delta: the DMA stored them in
        // register order (see rc_off), so each is one 64-B read straight into the tuple
        s = *reinterpret_cast<const f32x16*>(lse_s + 32 * h + 16 * hh);
        dp = *reinterpret_cast<const f32x16*>(del_s + 32 * h + 16 * hh);
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          s = mfma32(qa[ks], kf[ks], s);
          dp = mfma32(da[ks], vf[ks], dp);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      // first 16-row step's transposed fragments, read under the softmax (causal kernels only: the
      // full-attention build runs out of VGPRs with them)
      bf16x8_t dfr[NDB], qfr[NDB];
      if constexpr (CAUSAL) {
#pragma unroll
        for (int d = 0; d < NDB; ++d) {
          dfr[d] = tr_frag<HD>(Ds, 32 * h, d * 32, lane);
          qfr[d] = tr_frag<HD>(Qs, 32 * h, d * 32, lane);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      if (need_mask) {  // wave-uniform: one scalar branch around branch-free selects
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          const int row0 = 32 * h + 8 * gq + 4 * hh;  // rows of registers 4gq .. 4gq+3
          int sv[4] = {0, 0, 0, 0};
          if constexpr (DOC) {
            const int4 s4 = *reinterpret_cast<const int4*>(doc_s + row0);
            sv[0] = s4.x; sv[1] = s4.y; sv[2] = s4.z; sv[3] = s4.w;
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int qq = q0 + row0 + j;
            bool ok = qq < a.S && my_key < a.S;
            if constexpr (CAUSAL) ok = ok && my_key <= qq;
            if constexpr (DOC) ok = ok && my_key >= sv[j];
            s[4 * gq + j] = ok ? s[4 * gq + j] : -INFINITY;
          }
        }
      }
      float p[16], dsv[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float pv = fast_exp2(s[i] * a.scale_log2);
        p[i] = pv;
        dsv[i] = pv * dp[i];
      }
      bf16x8_t pb[2], sb[2];
      pb[0] = to_bf16x8(p);
      pb[1] = to_bf16x8(p + 8);
      sb[0] = to_bf16x8(dsv);
      sb[1] = to_bf16x8(dsv + 8);
      if constexpr (!CAUSAL) {
#pragma unroll
        for (int d = 0; d < NDB; ++d) {
          dfr[d] = tr_frag<HD>(Ds, 32 * h, d * 32, lane);
          qfr[d] = tr_frag<HD>(Qs, 32 * h, d * 32, lane);
        }
      }
      bf16x8_t dfr1[NDB], qfr1[NDB];  // second step's fragments land under the first step's MFMAs
#pragma unroll
      for (int d = 0; d < NDB; ++d) {
        dfr1[d] = tr_frag<HD>(Ds, 32 * h + 16, d * 32, lane);
        qfr1[d] = tr_frag<HD>(Qs, 32 * h + 16, d * 32, lane);
      }
      dvdk_step<NDB>(dv, dk, dfr, qfr, pb[0], sb[0]);
      dvdk_step<NDB>(dv, dk, dfr1, qfr1, pb[1], sb[1]);
    }
  };
  for (int t = 0; t < ntiles; t += NB) {
    step(std::integral_constant<int, 0>{}, t);
    if (t + 1 < ntiles) step(std::integral_constant<int, 1>{}, t + 1);
    if constexpr (NB >= 3)
      if (t + 2 < ntiles) step(std::integral_constant<int, 2 % NB>{}, t + 2);
    if constexpr (NB >= 4)
      if (t + 3 < ntiles) step(std::integral_constant<int, 3 % NB>{}, t + 3);
  }
  // ---- write dK (scaled), dV: lane = key, registers = d.  The asm MFMAs' results are read by
  //      compiler code below: 8-pass XDL D -> non-MFMA reader needs 12 wait states (unpadded by hipcc)
#pragma unroll
  for (int d = 0; d < NDB; ++d) asm volatile("s_nop 7\n\ts_nop 7" : "+a"(dk[d]), "+a"(dv[d]));
  if (my_key < a.S) {
    const long tok = (long)b * a.S + my_key;
    unsigned short* dkp = a.dk + tok * a.dk_st + (long)hk * HD;
    unsigned short* dvp = a.dv + tok * a.dv_st + (long)hk * HD;
    const float *cr = nullptr, *sr = nullptr;
    if (a.cos_t != nullptr) {
      const long p = a.rope_pos ? (long)a.rope_pos[tok] : tok % a.rope_S;
      cr = a.cos_t + p * (HD / 2);
      sr = a.sin_t + p * (HD / 2);
    }
    store_row<HD>(dkp, dk, a.scale, hh, cr, sr);
    store_row<HD>(dvp, dv, 1.f, hh, nullptr, nullptr);
  }
}

// =============================================================================================
// dQ
// =============================================================================================
template <int HD, bool CAUSAL, bool DOC>
__global__ __launch_bounds__(256, 2) void fa_bwd_dq_kernel(BwdArgs a) {
  constexpr int NKS = HD / 16;
  constexpr int NDB = HD / 32;
  constexpr int ROWB = HD * 2;
  constexpr int TILE = DQ_KB * ROWB;       // one K (or V) tile image
  constexpr int PPW = TILE / 1024 / 4;     // 1-KiB DMA pieces per wave per operand
  constexpr int SLOT = 2 * TILE;           // K (tr image) | V (row image)
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * SLOT];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const int nqb = (a.S + DQ_QB - 1) / DQ_QB;
  const int BH = a.B * a.Hq;
  int bh, qi;
  if (BH % 8) {
    bh = blockIdx.x % BH;
    qi = blockIdx.x / BH;
  } else {  // XCD-aware: XCD x walks heads [x*BH/8, (x+1)*BH/8), a head's q-blocks back to back
    const int x = blockIdx.x & 7, j = blockIdx.x >> 3;
    bh = x * (BH >> 3) + j / nqb;
    qi = j % nqb;
  }
  const int qblk = nqb - 1 - qi;  // heaviest first
  const int b = bh / a.Hq, hq = bh % a.Hq;
  const int hk = hq / (a.Hq / a.Hkv);
  const int q_row0 = qblk * DQ_QB + wave * 32;  // wave-uniform
  const int my_q = q_row0 + r;
  const int qc = min(my_q, a.S - 1);

  const unsigned short* Kp = a.k + b * a.k_sb + hk * a.k_sh;
  const unsigned short* Vp = a.v + b * a.v_sb + hk * a.v_sh;

#pragma unroll
  for (int i = 0; i < 2 * SLOT / 4096; ++i)
    *reinterpret_cast<uint4*>(smem + i * 4096 + tid * 16) = make_uint4(0, 0, 0, 0);

  // ---- Q and dO fragments (B operands of S^T = K Q^T and dP^T = V dO^T)
  bf16x8_t qf[NKS], df[NKS];
  {
    const unsigned short* Qp = a.q + b * a.q_sb + hq * a.q_sh + (long)qc * a.q_ss + 8 * hh;
    const unsigned short* Dp = a.dout + b * a.do_sb + hq * a.do_sh + (long)qc * a.do_ss + 8 * hh;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      qf[ks] = __builtin_bit_cast(bf16x8_t, gload16(Qp + 16 * ks));
      df[ks] = __builtin_bit_cast(bf16x8_t, gload16(Dp + 16 * ks));
    }
  }
  const long rc = ((long)b * a.Hq + hq) * a.S + qc;
  const float nlse2 = -a.lse[rc] * LOG2E;
  float dlt;
  if (a.o != nullptr) {  // delta of this lane's row: its 64 columns . dO, then the other half-wave's
    const unsigned short* Op = a.o + b * a.o_sb + hq * a.o_sh + (long)qc * a.o_ss + 8 * hh;
    float acc = 0.f;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const bf16x8_t of = __builtin_bit_cast(bf16x8_t, gload16(Op + 16 * ks));
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += (float)of[j] * (float)df[ks][j];
    }
    dlt = xor32_add(acc);
    if (hh == 0 && my_q < a.S) a.delta_w[rc] = dlt;
  } else {
    dlt = a.delta[rc];
  }
  if (hh == 0 && my_q < a.S) {
    a.rck_w[rc] = -a.lse[rc] / a.scale;
    a.rck_w[a.rc_n + rc] = -dlt;
  }
  // retire the loads here (a first use inside the loop would carry a per-iteration vmcnt(0) that
  // also drains the next tile's DMA)
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) asm volatile("" ::"v"(qf[ks]), "v"(df[ks]));
  asm volatile("" ::"v"(nlse2), "v"(dlt));

  f32x16 dq[NDB];
#pragma unroll
  for (int d = 0; d < NDB; ++d)
#pragma unroll
    for (int i = 0; i < 16; ++i) dq[d][i] = 0.f;

  const int kv_end = CAUSAL ? min(a.S, qblk * DQ_QB + DQ_QB) : a.S;
  const int ntiles = (kv_end + DQ_KB - 1) / DQ_KB;
  int my_start = 0, w_min = 0, w_max = 0, t0 = 0;
  if constexpr (DOC) {
    const int* ds = a.doc + (long)b * a.S;
    my_start = ds[qc];
    w_min = __builtin_amdgcn_readfirstlane(ds[min(q_row0, a.S - 1)]);
    w_max = __builtin_amdgcn_readfirstlane(ds[min(q_row0 + 31, a.S - 1)]);
    t0 = __builtin_amdgcn_readfirstlane(ds[min(qblk * DQ_QB, a.S - 1)]) / DQ_KB;
  }
  const int key_hi = CAUSAL ? qc : a.S - 1;  // last key this lane's row sees

  // ---- DMA ring (see the forward kernel): K as a tr image, V as a row image
  unsigned vk[PPW], vv[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int byte = (i * 4 + wave) * 1024 + lane * 16;
    const int row = byte / ROWB, pch = (byte % ROWB) >> 4;
    vk[i] = (unsigned)((row * a.k_ss + ((pch ^ swz_tr<HD>(row)) << 3)) * 2);
    vv[i] = (unsigned)((row * a.v_ss + ((pch ^ swz_row<HD>(row)) << 3)) * 2);
  }
  const unsigned lds0 = lds_addr(smem);
  // tiles are issued in order: the next one's key row and K / V pointers advance incrementally,
  // its ring slot is a template constant
  int ik0 = t0 * DQ_KB;
  const unsigned short* kc = Kp + (long)ik0 * a.k_ss;
  const unsigned short* vc = Vp + (long)ik0 * a.v_ss;
  const long k_step = (long)DQ_KB * a.k_ss, v_step = (long)DQ_KB * a.v_ss;
  auto issue = [&](auto slot_c) __attribute__((always_inline)) {
    constexpr int SLC = decltype(slot_c)::value;
    const int nk = min(DQ_KB, a.S - ik0);
    i32x4_t rk = buf_rsrc(kc, (unsigned)(((nk - 1) * a.k_ss + HD) * 2));
    i32x4_t rv = buf_rsrc(vc, (unsigned)(((nk - 1) * a.v_ss + HD) * 2));
    // descriptor SGPRs may come from v_readfirstlane: VALU-written SGPR -> VMEM read needs 5
    // wait states, which hipcc does not pad into the asm below (guide §5.7 item 2)
    asm volatile("s_nop 4" : "+s"(rk), "+s"(rv));
    const unsigned slot = lds0 + (unsigned)(SLC * SLOT) + wave * 1024;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      buf_dma16(rk, vk[i], slot + i * 4096);
      buf_dma16(rv, vv[i], slot + TILE + i * 4096);
    }
    ik0 += DQ_KB;
    kc += k_step;
    vc += v_step;
  };

  auto tile = [&](bool need_mask, const unsigned char* Ks, const unsigned char* Vs, int kv0)
                  __attribute__((always_inline)) {
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      // ---- S^T = K Q^T, dP^T = V dO^T   (key on regs, q on lane)
      f32x16 s, dp;
#pragma unroll
      for (int i = 0; i < 16; ++i) s[i] = dp[i] = 0.f;
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        s = mfma32(lds_read_b128(Ks, tr_off<HD>(kb * 32 + r, 2 * ks + hh)), qf[ks], s);
        dp = mfma32(lds_read_b128(Vs, row_off<HD>(kb * 32 + r, 2 * ks + hh)), df[ks], dp);
      }
      if (need_mask) {  // wave-uniform: a scalar branch around branch-free selects
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int key = kv0 + kb * 32 + acc_row(i, hh);
          bool ok = key <= key_hi;
          if constexpr (DOC) ok = ok && key >= my_start;
          s[i] = ok ? s[i] : -INFINITY;
        }
      }
      float dsv[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) dsv[i] = fast_exp2(__builtin_fmaf(s[i], a.scale_log2, nlse2)) * (dp[i] - dlt);
      // ---- dQ^T += K^T dS^T   (sum over keys = the registers of dS^T)
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const bf16x8_t sbf = to_bf16x8(dsv + 8 * st);
#pragma unroll
        for (int d = 0; d < NDB; ++d) dq[d] = mfma32(tr_frag<HD>(Ks, kb * 32 + 16 * st, d * 32, lane), sbf, dq[d]);
      }
    }
  };

  __syncthreads();  // ring zeroed before any DMA lands in it
  auto step = [&](auto slot_c, int t) __attribute__((always_inline)) {
    constexpr int SL = decltype(slot_c)::value;
    vm_wait_n<0>();
    __builtin_amdgcn_s_barrier();
    if (t + 1 < ntiles) issue(std::integral_constant<int, 1 - SL>{});
    const int kv0 = t * DQ_KB;
    bool live = true;
    if constexpr (CAUSAL) live = kv0 <= q_row0 + 31;
    if constexpr (DOC) live = live && kv0 + DQ_KB > w_min;
    if (live) {
      const bool need_mask =
          (CAUSAL && kv0 + DQ_KB - 1 > q_row0) || (kv0 + DQ_KB > a.S) || (DOC && kv0 < w_max);
      tile(need_mask, smem + SL * SLOT, smem + SL * SLOT + TILE, kv0);
    }
  };
  if (t0 < ntiles) issue(std::integral_constant<int, 0>{});
  for (int t = t0; t < ntiles; t += 2) {
    step(std::integral_constant<int, 0>{}, t);
    if (t + 1 < ntiles) step(std::integral_constant<int, 1>{}, t + 1);
  }
  // ---- dQ = scale * (dQ^T)^T: lane = q row, registers = d
  if (my_q < a.S) {
    const long tok = (long)b * a.S + my_q;
    const float *cr = nullptr, *sr = nullptr;
    if (a.cos_t != nullptr) {
      const long p = a.rope_pos ? (long)a.rope_pos[tok] : tok % a.rope_S;
      cr = a.cos_t + p * (HD / 2);
      sr = a.sin_t + p * (HD / 2);
    }
    store_row<HD>(a.dq + tok * a.dq_st + (long)hq * HD, dq, a.scale, hh, cr, sr);
  }
}

template <int HD, bool CAUSAL, bool DOC>
void launch_bwd(const BwdArgs& a, hipStream_t s, bool do_dq, bool do_dkv) {
  if (do_dq) {
    const int nqb = (a.S + DQ_QB - 1) / DQ_QB;
    hipLaunchKernelGGL((fa_bwd_dq_kernel<HD, CAUSAL, DOC>), dim3((unsigned)(a.B * a.Hq * nqb)), dim3(256), 0, s, a);
  }
  if (do_dkv) {
    const int nkb = (a.S + KV_KB - 1) / KV_KB;
    hipLaunchKernelGGL((fa_bwd_dkv_kernel<HD, CAUSAL, DOC>), dim3((unsigned)(a.B * a.Hkv * nkb)), dim3(256), 0, s,
                       a);
  }
}

void dispatch_bwd(const BwdArgs& a, int D, bool causal, bool doc, hipStream_t s, bool do_dq = true,
                  bool do_dkv = true) {
  if (doc) {
    if (D == 128) launch_bwd<128, true, true>(a, s, do_dq, do_dkv);
    else launch_bwd<64, true, true>(a, s, do_dq, do_dkv);
  } else if (D == 128) {
    if (causal) launch_bwd<128, true, false>(a, s, do_dq, do_dkv);
    else launch_bwd<128, false, false>(a, s, do_dq, do_dkv);
  } else {
    if (causal) launch_bwd<64, true, false>(a, s, do_dq, do_dkv);
    else launch_bwd<64, false, false>(a, s, do_dq, do_dkv);
  }
}

BwdArgs make_args(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                  const at::Tensor& lse, const at::Tensor& delta, at::Tensor& dq, at::Tensor& dk, at::Tensor& dv,
                  double scale) {
  return BwdArgs{bf_ptr(q), bf_ptr(k), bf_ptr(v), bf_ptr(dout), lse.data_ptr<float>(), delta.data_ptr<float>(),
                 bf_mut(dq), bf_mut(dk), bf_mut(dv), (int)q.size(0), (int)q.size(1), (int)q.size(2),
                 (int)k.size(2), q.stride(0), q.stride(1), q.stride(2), k.stride(0), k.stride(1), k.stride(2),
                 v.stride(0), v.stride(1), v.stride(2), dout.stride(0), dout.stride(1), dout.stride(2),
                 (float)scale, (float)(scale * 1.4426950408889634), nullptr,
                 (long)dq.size(2) * dq.size(3), (long)dk.size(2) * dk.size(3), (long)dv.size(2) * dv.size(3),
                 nullptr, nullptr, nullptr, 0, nullptr, 0, 0, 0, nullptr, nullptr, 0};
}

// the dQ kernel's [2, B*Hq*S] row-constant output for the dK/dV kernel (BwdArgs::rck_w)
at::Tensor row_consts(BwdArgs& a, const at::Tensor& lse) {
  auto rck = at::empty({2 * lse.numel()}, lse.options());
  a.rck_w = rck.data_ptr<float>();
  a.rc_n = lse.numel();
  return rck;
}

}  // namespace

std::tuple<at::Tensor, at::Tensor, at::Tensor> flash_attn_bwd(const at::Tensor& dout, const at::Tensor& q,
                                                              const at::Tensor& k, const at::Tensor& v,
                                                              const at::Tensor& o, const at::Tensor& lse,
                                                              double scale, bool causal,
                                                              const c10::optional<at::Tensor>& doc_start) {
  LLMCTL_CHECK(q.dim() == 4 && k.dim() == 4 && v.dim() == 4 && o.dim() == 4 && dout.dim() == 4,
               "flash_attn_bwd: [B,S,H,D] tensors");
  const int B = q.size(0), S = q.size(1), Hq = q.size(2), D = q.size(3);
  const int Hkv = k.size(2);
  LLMCTL_CHECK(D == 64 || D == 128, "head_dim must be 64 or 128");
  LLMCTL_CHECK(Hkv > 0 && Hq % Hkv == 0, "Hq must be a multiple of Hkv");
  LLMCTL_CHECK(dout.sizes() == q.sizes() && o.sizes() == q.sizes() && k.sizes() == v.sizes() && k.size(0) == B &&
                   k.size(1) == S && k.size(3) == D,
               "shape mismatch");
  LLMCTL_CHECK(lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.numel() == (long)B * Hq * S,
               "lse must be contiguous fp32 [B,Hq,S]");
  for (const at::Tensor* t : {&dout, &q, &k, &v, &o})
    LLMCTL_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 && t->stride(3) == 1 && t->stride(0) % 8 == 0 &&
                     t->stride(1) % 8 == 0 && t->stride(2) % 8 == 0 &&
                     (reinterpret_cast<uintptr_t>(t->data_ptr()) & 15) == 0,
                 "flash_attn_bwd: bf16, d-contiguous, 16-B aligned rows");
  const c10::DeviceGuard g(q.device());
  auto delta = at::empty({B, Hq, S}, q.options().dtype(at::kFloat));
  auto dq = at::empty({B, S, Hq, D}, q.options());
  auto dk = at::empty({B, S, Hkv, D}, q.options());
  auto dv = at::empty({B, S, Hkv, D}, q.options());
  if ((long)B * S * Hq == 0) return {dq, dk, dv};
  auto s = stream();
  BwdArgs a = make_args(dout, q, k, v, lse, delta, dq, dk, dv, scale);
  a.o = bf_ptr(o);
  a.o_sb = o.stride(0);
  a.o_ss = o.stride(1);
  a.o_sh = o.stride(2);
  a.delta_w = delta.data_ptr<float>();
  auto rck = row_consts(a, lse);
  bool doc = false;
  if (doc_start.has_value() && doc_start->defined()) {
    const at::Tensor& ds = *doc_start;
    LLMCTL_CHECK(causal && ds.is_cuda() && ds.scalar_type() == at::kInt && ds.is_contiguous() && ds.dim() == 2 &&
                     ds.size(0) == B && ds.size(1) == S,
                 "flash_attn_bwd: doc_start must be contiguous int32 [B,S] (causal)");
    a.doc = ds.data_ptr<int>();
    doc = true;
  }
  dispatch_bwd(a, D, causal, doc, s);
  return {dq, dk, dv};
}

// Attention backward with the RoPE backward fused into the dQ / dK stores: returns the gradient of
// the QKV projection output dqkv [B*S, (Hq + 2 Hkv) * D] directly (dq / dk rotated back by their
// positions, dv copied), the layout ``rope_qkv`` split the projection from.  cos / sin: fp32
// [>= max position, D/2]; positions: int32 [B*S] or none (position = token % seq_len).
at::Tensor flash_attn_bwd_qkv(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                              const at::Tensor& o, const at::Tensor& lse, double scale, bool causal,
                              const c10::optional<at::Tensor>& doc_start, const at::Tensor& cos_t,
                              const at::Tensor& sin_t, const c10::optional<at::Tensor>& positions, int64_t seq_len) {
  LLMCTL_CHECK(q.dim() == 4 && k.dim() == 4 && v.dim() == 4 && o.dim() == 4 && dout.dim() == 4,
               "flash_attn_bwd_qkv: [B,S,H,D] tensors");
  const int B = q.size(0), S = q.size(1), Hq = q.size(2), D = q.size(3);
  const int Hkv = k.size(2);
  LLMCTL_CHECK(D == 64 || D == 128, "head_dim must be 64 or 128");
  LLMCTL_CHECK(Hkv > 0 && Hq % Hkv == 0, "Hq must be a multiple of Hkv");
  LLMCTL_CHECK(dout.sizes() == q.sizes() && o.sizes() == q.sizes() && k.sizes() == v.sizes() && k.size(0) == B &&
                   k.size(1) == S && k.size(3) == D,
               "shape mismatch");
  LLMCTL_CHECK(lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.numel() == (long)B * Hq * S,
               "lse must be contiguous fp32 [B,Hq,S]");
  for (const at::Tensor* t : {&dout, &q, &k, &v, &o})
    LLMCTL_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 && t->stride(3) == 1 && t->stride(0) % 8 == 0 &&
                     t->stride(1) % 8 == 0 && t->stride(2) % 8 == 0 &&
                     (reinterpret_cast<uintptr_t>(t->data_ptr()) & 15) == 0,
                 "flash_attn_bwd_qkv: bf16, d-contiguous, 16-B aligned rows");
  LLMCTL_CHECK(cos_t.is_cuda() && sin_t.is_cuda() && cos_t.scalar_type() == at::kFloat &&
                   sin_t.scalar_type() == at::kFloat && cos_t.is_contiguous() && sin_t.is_contiguous() &&
                   cos_t.dim() == 2 && cos_t.size(1) == D / 2 && sin_t.sizes() == cos_t.sizes(),
               "flash_attn_bwd_qkv: cos/sin fp32 contiguous [P, D/2]");
  const bool has_pos = positions.has_value() && positions->defined();
  if (has_pos) {
    LLMCTL_CHECK(positions->is_cuda() && positions->scalar_type() == at::kInt && positions->is_contiguous() &&
                     positions->numel() == (long)B * S,
                 "flash_attn_bwd_qkv: positions int32 [B*S]");
  } else {
    LLMCTL_CHECK(seq_len > 0 && seq_len <= cos_t.size(0), "flash_attn_bwd_qkv: seq_len within the tables");
  }
  const c10::DeviceGuard g(q.device());
  const long W = (long)(Hq + 2 * Hkv) * D;
  auto dqkv = at::empty({(long)B * S, W}, q.options());
  if ((long)B * S * Hq == 0) return dqkv;
  auto delta = at::empty({B, Hq, S}, q.options().dtype(at::kFloat));
  auto s = stream();
  unsigned short* base = bf_mut(dqkv);
  BwdArgs a{bf_ptr(q), bf_ptr(k), bf_ptr(v), bf_ptr(dout), lse.data_ptr<float>(), delta.data_ptr<float>(),
            base, base + (long)Hq * D, base + (long)(Hq + Hkv) * D, B, S, Hq, Hkv,
            q.stride(0), q.stride(1), q.stride(2), k.stride(0), k.stride(1), k.stride(2),
            v.stride(0), v.stride(1), v.stride(2), dout.stride(0), dout.stride(1), dout.stride(2),
            (float)scale, (float)(scale * 1.4426950408889634), nullptr, W, W, W,
            cos_t.data_ptr<float>(), sin_t.data_ptr<float>(), has_pos ? positions->data_ptr<int>() : nullptr,
            (int)(has_pos ? 1 : seq_len), bf_ptr(o), o.stride(0), o.stride(1), o.stride(2),
            delta.data_ptr<float>(), nullptr, 0};
  auto rck = row_consts(a, lse);
  bool doc = false;
  if (doc_start.has_value() && doc_start->defined()) {
    const at::Tensor& ds = *doc_start;
    LLMCTL_CHECK(causal && ds.is_cuda() && ds.scalar_type() == at::kInt && ds.is_contiguous() && ds.dim() == 2 &&
                     ds.size(0) == B && ds.size(1) == S,
                 "flash_attn_bwd_qkv: doc_start must be contiguous int32 [B,S] (causal)");
    a.doc = ds.data_ptr<int>();
    doc = true;
  }
  dispatch_bwd(a, D, causal, doc, s);
  return dqkv;
}

// timing-only entry for tools/attn_ablate.py (causal, no documents): abl 0 = both kernels,
// 1 = dK/dV kernel only (its row constants prepared by two small torch ops), 2 = dQ kernel only.
// ``delta`` is taken as given.
void fa_bwd_ablate(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                   const at::Tensor& delta, const at::Tensor& lse, at::Tensor& dq, at::Tensor& dk, at::Tensor& dv,
                   int64_t abl) {
  const int D = q.size(3);
  LLMCTL_CHECK(D == 64 || D == 128, "fa_bwd_ablate: head_dim 64 or 128");
  LLMCTL_CHECK(dq.scalar_type() == at::kBFloat16 && dq.sizes() == q.sizes() && dk.sizes() == k.sizes() &&
                   dv.sizes() == k.sizes() && delta.numel() == lse.numel(),
               "fa_bwd_ablate: bf16 dq/dk/dv, fp32 delta");
  const c10::DeviceGuard g(q.device());
  const double scale = 1.0 / std::sqrt((double)D);
  BwdArgs a = make_args(dout, q, k, v, lse, delta, dq, dk, dv, scale);
  auto rck = row_consts(a, lse);
  if (abl == 1) {  // no dQ kernel to write them
    rck.narrow(0, 0, lse.numel()).copy_(lse.reshape(-1) * (-1.0 / scale));
    rck.narrow(0, lse.numel(), lse.numel()).copy_(-delta.reshape(-1));
  }
  dispatch_bwd(a, D, true, false, stream(), abl != 1, abl != 2);
}

TORCH_LIBRARY_IMPL(llmctl, CUDA, m) {
  m.impl("flash_attn_bwd", &flash_attn_bwd);
  m.impl("flash_attn_bwd_qkv", &flash_attn_bwd_qkv);
  m.impl("fa_bwd_ablate", &fa_bwd_ablate);
}

}  // namespace llmctl
