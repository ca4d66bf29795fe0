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
#include <cstdlib>
#include <map>
#include <mutex>

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
  // diagnostic timeline (fa_bwd_ablate abl 6 only): per workgroup 8 x u64, see the pipelined kernel
  unsigned long long* stamps = nullptr;
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

// ---------------------------------------------------------------------------------------------
// dK / dV, software-pipelined (round 3).  Same work decomposition, LDS ring and register-resident
// K / V as fa_bwd_dkv_kernel, but the per-tile program is reordered so the matrix pipe is never
// idle behind the softmax VALU of the same wave.  PMC of the kernel above (B12 S2048 H32 D128,
// profiles/attn_pmc_r3.txt): MFMA busy 28 %, the wave stalled on issue 46 % and on waits 21 % of
// its cycles — one wave per SIMD, every phase (fragment reads -> S/dP MFMAs -> softmax ->
// dV/dK MFMAs) serialised behind the previous one.  Here, per 64-row tile (halves 0 / 1):
//     R0  S0/dP0 (16 MFMA)  R1  X: S1/dP1 (16 MFMA) || softmax(half 0)
//     T0  Y: dV/dK(half 0) (16 MFMA) || softmax(half 1)   T1  dV/dK(half 1) (16 MFMA)
// where R = Q / dO fragment + row-constant reads, T = transposed fragment reads.  X and Y are
// inline-asm statements of two MFMAs plus the softmax of two scores (p = exp2(c s'),
// ds = p dp', bf16 pairs): asm volatile keeps their order, so each MFMA's 32 issue cycles hide
// ~8 VALU instructions of the other half instead of the VALU waiting for the pipe to drain.
// Hazards (hipcc pads none inside asm): the exp results are read two instructions after their
// v_exp (trans -> VALU), the S/dP results are read by VALU >= 2 MFMAs after the last MFMA that
// wrote them, and the packed P / dS words are read by MFMAs >= 3 statements after their cvt.
using s2_t = __attribute__((ext_vector_type(2))) unsigned int;

__device__ __forceinline__ bf16x8_t words8(unsigned w0, unsigned w1, unsigned w2, unsigned w3) {
  using u4 = __attribute__((ext_vector_type(4))) unsigned;
  return __builtin_bit_cast(bf16x8_t, u4{w0, w1, w2, w3});
}

__device__ __forceinline__ void mfma_v(f32x16& acc, bf16x8_t a, bf16x8_t b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "a"(b) : "memory");
}

// X: acc_s += a_s b_s, acc_d += a_d b_d (VGPR accumulators; b_s / b_d = the wave's K / V
// fragments, AGPR-resident) || softmax of (s0, s1) with dp (d0, d1).  The "memory" clobber pins the
// fragment reads placed between the statements (the next phase's operands stream in under these
// MFMAs instead of being hoisted into one burst).
__device__ __forceinline__ void x_step(f32x16& acc_s, f32x16& acc_d, bf16x8_t a_s, bf16x8_t b_s, bf16x8_t a_d,
                                       bf16x8_t b_d, float s0, float s1, float d0, float d1, float c, unsigned& pw,
                                       unsigned& dw) {
  float t0, t1, p0, p1;
  asm volatile(
      "v_mul_f32 %[t0], %[c], %[s0]\n\t"
      "v_mul_f32 %[t1], %[c], %[s1]\n\t"
      "v_mfma_f32_32x32x16_bf16 %[as], %[xs], %[ys], %[as]\n\t"
      "v_exp_f32 %[p0], %[t0]\n\t"
      "v_exp_f32 %[p1], %[t1]\n\t"
      "v_mfma_f32_32x32x16_bf16 %[ad], %[xd], %[yd], %[ad]\n\t"
      "v_mul_f32 %[t0], %[p0], %[d0]\n\t"
      "v_mul_f32 %[t1], %[p1], %[d1]\n\t"
      "v_cvt_pk_bf16_f32 %[pw], %[p0], %[p1]\n\t"
      "v_cvt_pk_bf16_f32 %[dw], %[t0], %[t1]"
      : [as] "+v"(acc_s), [ad] "+v"(acc_d), [t0] "=&v"(t0), [t1] "=&v"(t1), [p0] "=&v"(p0), [p1] "=&v"(p1),
        [pw] "=&v"(pw), [dw] "=&v"(dw)
      : [xs] "v"(a_s), [ys] "a"(b_s), [xd] "v"(a_d), [yd] "a"(b_d), [s0] "v"(s0), [s1] "v"(s1), [d0] "v"(d0),
        [d1] "v"(d1), [c] "s"(c)
      : "memory");
}

// Y: dv += da p, dk += qa ds (AGPR accumulators) || softmax of (s0, s1) with dp (d0, d1)
__device__ __forceinline__ void y_step(f32x16& dv, f32x16& dk, bf16x8_t da, bf16x8_t qa, bf16x8_t p, bf16x8_t ds,
                                       float s0, float s1, float d0, float d1, float c, unsigned& pw, unsigned& dw) {
  float t0, t1, p0, p1;
  asm volatile(
      "v_mul_f32 %[t0], %[c], %[s0]\n\t"
      "v_mul_f32 %[t1], %[c], %[s1]\n\t"
      "v_mfma_f32_32x32x16_bf16 %[dv], %[da], %[p], %[dv]\n\t"
      "v_exp_f32 %[p0], %[t0]\n\t"
      "v_exp_f32 %[p1], %[t1]\n\t"
      "v_mfma_f32_32x32x16_bf16 %[dk], %[qa], %[ds], %[dk]\n\t"
      "v_mul_f32 %[t0], %[p0], %[d0]\n\t"
      "v_mul_f32 %[t1], %[p1], %[d1]\n\t"
      "v_cvt_pk_bf16_f32 %[pw], %[p0], %[p1]\n\t"
      "v_cvt_pk_bf16_f32 %[dw], %[t0], %[t1]"
      : [dv] "+a"(dv), [dk] "+a"(dk), [t0] "=&v"(t0), [t1] "=&v"(t1), [p0] "=&v"(p0), [p1] "=&v"(p1),
        [pw] "=&v"(pw), [dw] "=&v"(dw)
      : [da] "v"(da), [qa] "v"(qa), [p] "v"(p), [ds] "v"(ds), [s0] "v"(s0), [s1] "v"(s1), [d0] "v"(d0),
        [d1] "v"(d1), [c] "s"(c)
      : "memory");
}

// AGPR accumulator tuple -> VGPR copy for an epilogue, and in-place zeroing through the matrix pipe
// (0 * 0 + 0): the compiler never writes the dK / dV AGPRs itself (a C++ write made hipcc keep them
// in VGPRs and copy them around every asm use)
__device__ __forceinline__ f32x16 acc_copy(const f32x16& acc) {
  // plain reads (v_accvgpr_read); the asm statement only orders them and keeps the stores after it
  f32x16 out = acc;
  asm volatile("" : "+v"(out)::"memory");
  return out;
}
__device__ __forceinline__ void acc_zero(f32x16& acc) {  // in place ("+a": no second register set)
  const bf16x8_t z = {};  // MFMA A / B take no inline constants, C does
  // z was just written by a VALU v_mov: the MFMA must not read it within 2 wait states (hipcc pads
  // none inside asm; without the nop the first zeroing MFMA read stale register contents and seeded
  // dK with garbage / NaN now and then)
  asm volatile("s_nop 2\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %1, 0" : "+a"(acc) : "v"(z));
}

// dV / dK of one 16-row step with no softmax work beside it (the previous tile's second half)
__device__ __forceinline__ void z_step(f32x16& dv, f32x16& dk, bf16x8_t da, bf16x8_t qa, bf16x8_t p, bf16x8_t ds) {
  asm volatile(
      "v_mfma_f32_32x32x16_bf16 %[dv], %[da], %[p], %[dv]\n\t"
      "v_mfma_f32_32x32x16_bf16 %[dk], %[qa], %[ds], %[dk]"
      : [dv] "+a"(dv), [dk] "+a"(dk)
      : [da] "v"(da), [qa] "v"(qa), [p] "v"(p), [ds] "v"(ds)
      : "memory");
}

template <int HD, bool CAUSAL, bool DOC, bool STAMP = false>
__global__ __launch_bounds__(256, 1) void fa_bwd_dkv_pipe_kernel(BwdArgs a) {
  static_assert(HD == 128 && CAUSAL, "pipelined dK/dV kernel: causal, head_dim 128");
  constexpr int NKS = HD / 16;
  constexpr int NDB = HD / 32;
  constexpr int ROWB = HD * 2;
  constexpr int TILE_B = KV_QT * ROWB;
  constexpr int NP = TILE_B / 1024 / 4;
  constexpr int RC_B = KV_QT * 4;
  constexpr int BUF_B = 2 * TILE_B + 4 * RC_B;  // Q | dO | lse | delta | doc | (pad)
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * BUF_B];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;
  // STAMP: [0] entry, [1] HW_ID | XCC_ID << 32, [2] prologue done, [3] tile loop done, [4] epilogue
  // stores retired, [5] tiles (constant-rate s_memrealtime, 100 MHz; workgroup's thread 0)
  auto stamp = [&](int i) __attribute__((always_inline)) {
    if constexpr (STAMP) {
      if (tid == 0) a.stamps[blockIdx.x * 8 + i] = __builtin_amdgcn_s_memrealtime();
    }
  };
  stamp(0);
  if constexpr (STAMP) {
    if (tid == 0)
      a.stamps[blockIdx.x * 8 + 1] = (unsigned long long)(unsigned)__builtin_amdgcn_s_getreg(63492) |
                                     ((unsigned long long)(unsigned)__builtin_amdgcn_s_getreg(63508) << 32);
  }
  const int nkb = (a.S + KV_KB - 1) / KV_KB;
  const int BH = a.B * a.Hkv;
  int bh, kblk;
  if (BH % 8) {
    bh = blockIdx.x % BH;
    kblk = blockIdx.x / BH;
  } else {
    const int x = blockIdx.x & 7, j = blockIdx.x >> 3;
    bh = x * (BH >> 3) + j / nkb;
    kblk = j % nkb;
  }
  const int b = bh / a.Hkv, hk = bh % a.Hkv;
  const int group = a.Hq / a.Hkv;
  const int k0 = kblk * KV_KB;
  const int wkey0 = k0 + wave * 32;
  const int my_key = wkey0 + r;

  if (a.S % KV_QT) {  // partial tiles: rows past S stay unwritten by the DMA and must read finite
#pragma unroll
    for (int i = 0; i < 2 * BUF_B / 4096; ++i)
      *reinterpret_cast<uint4*>(smem + i * 4096 + tid * 16) = make_uint4(0, 0, 0, 0);
    if (tid < (2 * BUF_B % 4096) / 16)
      *reinterpret_cast<uint4*>(smem + (2 * BUF_B / 4096) * 4096 + tid * 16) = make_uint4(0, 0, 0, 0);
    __syncthreads();
  }

  const unsigned lds0 = lds_addr(smem);

  f32x16 dk[NDB], dv[NDB];
#pragma unroll
  for (int d = 0; d < NDB; ++d)
#pragma unroll
    for (int i = 0; i < 16; ++i) dk[d][i] = dv[d][i] = 0.f;

  const int q_start = CAUSAL ? k0 : 0;
  int q_end = a.S;
  if constexpr (DOC) {
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
  unsigned vq[NP], vd[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int byte = (i * 4 + wave) * 1024 + lane * 16;
    const int row = byte / ROWB;
    const int lch = ((byte % ROWB) >> 4) ^ swz_tr<HD>(row);
    vq[i] = (unsigned)((row * a.q_ss + lch * 8) * 2);
    vd[i] = (unsigned)((row * a.do_ss + lch * 8) * 2);
  }
  const float* rc_src = a.rck_w + (wave == 1 ? a.rc_n : 0);
  const unsigned rc_off =
      (DOC && wave == 2) ? lane * 4
                         : (unsigned)((32 * (lane >> 5) + 8 * ((lane >> 2) & 3) + 4 * ((lane >> 4) & 1) + (lane & 3)) * 4);
  int iq0 = q_start;
  const unsigned short* qh = a.q + b * a.q_sb + (long)(hk * group) * a.q_sh;
  const unsigned short* dh = a.dout + b * a.do_sb + (long)(hk * group) * a.do_sh;
  const float* rh = rc_src + ((long)b * a.Hq + hk * group) * a.S;
  const unsigned short* qc = qh + (long)q_start * a.q_ss;
  const unsigned short* dc = dh + (long)q_start * a.do_ss;
  const long q_step = (long)KV_QT * a.q_ss, d_step = (long)KV_QT * a.do_ss;
  auto issue = [&](auto slot_c) __attribute__((always_inline)) {
    constexpr int SLC = decltype(slot_c)::value;
    const int nr = min(KV_QT, a.S - iq0);
    i32x4_t rq = buf_rsrc(qc, (unsigned)(((nr - 1) * a.q_ss + HD) * 2));
    i32x4_t rd = buf_rsrc(dc, (unsigned)(((nr - 1) * a.do_ss + HD) * 2));
    i32x4_t rr = (DOC && wave == 2) ? buf_rsrc(a.doc + (long)b * a.S + iq0, (unsigned)(nr * 4))
                                    : buf_rsrc(rh + iq0, (unsigned)(nr * 4));
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
    if (iq0 >= q_end) {
      iq0 = q_start;
      qh += a.q_sh;
      dh += a.do_sh;
      rh += a.S;
      qc = qh + (long)q_start * a.q_ss;
      dc = dh + (long)q_start * a.do_ss;
    }
  };

  const float c = a.scale_log2;
  // masked scores of half h (rows 32h..32h+31 of the tile starting at q0): -inf where invisible
  auto apply_mask = [&](f32x16& s, int h, int q0, const int* doc_s) __attribute__((always_inline)) {
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      const int row0 = 32 * h + 8 * gq + 4 * hh;
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
  };

  // prologue: tile 0's DMA first, the K / V fragments under it (both latencies overlap), one wait
  if (ntiles > 0) issue(std::integral_constant<int, 0>{});
  // the wave's K / V fragments, loaded straight into AGPRs (every use is an MFMA B operand with an
  // "a" constraint, so they never occupy VGPRs and need no per-use copy)
  bf16x8_t kf[NKS], vf[NKS];
  {
    const int kc = min(my_key, a.S - 1);
    const unsigned short* Kp = a.k + b * a.k_sb + hk * a.k_sh + (long)kc * a.k_ss + 8 * hh;
    const unsigned short* Vp = a.v + b * a.v_sb + hk * a.v_sh + (long)kc * a.v_ss + 8 * hh;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      asm volatile("global_load_dwordx4 %0, %1, off" : "=a"(kf[ks]) : "v"(Kp + 16 * ks) : "memory");
      asm volatile("global_load_dwordx4 %0, %1, off" : "=a"(vf[ks]) : "v"(Vp + 16 * ks) : "memory");
    }
  }
  vm_wait_n<0>();
  __builtin_amdgcn_s_barrier();
  stamp(2);
  if (ntiles > 1) issue(std::integral_constant<int, 1>{});
  int qi = 0;
  auto tile = [&](auto slot_c, int t) __attribute__((always_inline)) {
    constexpr int SL = decltype(slot_c)::value;
    const int q0 = q_start + qi * KV_QT;
    if (++qi == nq) qi = 0;
    const bool live = !(CAUSAL && wkey0 > q0 + KV_QT - 1);
    const unsigned char* Qs = smem + SL * BUF_B;
    const unsigned char* Ds = Qs + TILE_B;
    const float* lse_s = reinterpret_cast<const float*>(Ds + TILE_B);
    const float* del_s = lse_s + KV_QT;
    const int* doc_s = reinterpret_cast<const int*>(del_s + KV_QT);
    if (!live) return;
    // ---- R0: row constants first (the first MFMA's accumulators), then the fragments
    f32x16 s0 = *reinterpret_cast<const f32x16*>(lse_s + 16 * hh);
    f32x16 p0 = *reinterpret_cast<const f32x16*>(del_s + 16 * hh);
    bf16x8_t qa[NKS], da[NKS];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      qa[ks] = lds_read_b128(Qs, tr_off<HD>(r, 2 * ks + hh));
      da[ks] = lds_read_b128(Ds, tr_off<HD>(r, 2 * ks + hh));
    }
    const bool need_mask = DOC || (CAUSAL && wkey0 + 31 > q0) || (q0 + KV_QT > a.S) || (wkey0 + 31 >= a.S);
    // ---- S0 / dP0
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      mfma_v(s0, qa[ks], kf[ks]);
      mfma_v(p0, da[ks], vf[ks]);
    }
    // ---- R1, then X: S1 / dP1 || softmax of half 0, with the half-0 transposed fragments (T0)
    //      read two per statement
    f32x16 s1 = *reinterpret_cast<const f32x16*>(lse_s + 32 + 16 * hh);
    f32x16 p1 = *reinterpret_cast<const f32x16*>(del_s + 32 + 16 * hh);
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      qa[ks] = lds_read_b128(Qs, tr_off<HD>(32 + r, 2 * ks + hh));
      da[ks] = lds_read_b128(Ds, tr_off<HD>(32 + r, 2 * ks + hh));
    }
    if (need_mask) apply_mask(s0, 0, q0, doc_s);
    unsigned pw0[8], dw0[8];
    bf16x8_t td[2][NDB], tq[2][NDB];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      x_step(s1, p1, qa[ks], kf[ks], da[ks], vf[ks], s0[2 * ks], s0[2 * ks + 1], p0[2 * ks], p0[2 * ks + 1], c, pw0[ks],
             dw0[ks]);
      const int st = ks >> 2, d = ks & 3;
      td[st][d] = tr_frag<HD>(Ds, 16 * st, d * 32, lane);
      tq[st][d] = tr_frag<HD>(Qs, 16 * st, d * 32, lane);
    }
    // ---- Y: dV / dK (half 0) || softmax of half 1, with the half-1 transposed fragments (T1)
    if (need_mask) apply_mask(s1, 1, q0, doc_s);
    unsigned pw1[8], dw1[8];
    bf16x8_t cd[2][NDB], cq[2][NDB];
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const bf16x8_t pb = words8(pw0[4 * st], pw0[4 * st + 1], pw0[4 * st + 2], pw0[4 * st + 3]);
      const bf16x8_t sb = words8(dw0[4 * st], dw0[4 * st + 1], dw0[4 * st + 2], dw0[4 * st + 3]);
#pragma unroll
      for (int d = 0; d < NDB; ++d) {
        const int i = 4 * st + d;
        y_step(dv[d], dk[d], td[st][d], tq[st][d], pb, sb, s1[2 * i], s1[2 * i + 1], p1[2 * i], p1[2 * i + 1], c,
               pw1[i], dw1[i]);
        cd[st][d] = tr_frag<HD>(Ds, 32 + 16 * st, d * 32, lane);
        cq[st][d] = tr_frag<HD>(Qs, 32 + 16 * st, d * 32, lane);
      }
    }
    // ---- dV / dK (half 1): MFMAs only; the pipe drains into the barrier
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const bf16x8_t pb = words8(pw1[4 * st], pw1[4 * st + 1], pw1[4 * st + 2], pw1[4 * st + 3]);
      const bf16x8_t sb = words8(dw1[4 * st], dw1[4 * st + 1], dw1[4 * st + 2], dw1[4 * st + 3]);
#pragma unroll
      for (int d = 0; d < NDB; ++d) z_step(dv[d], dk[d], cd[st][d], cq[st][d], pb, sb);
    }
  };
  // after each tile: every wave's reads of its slot retired and tile t+1's DMA landed ->
  // barrier, then the slot takes tile t+2
  auto advance = [&](auto slot_c, int t) __attribute__((always_inline)) {
    constexpr int SL = decltype(slot_c)::value;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    vm_wait_n<0>();
    __builtin_amdgcn_s_barrier();
    if (t + 2 < ntiles) issue(std::integral_constant<int, SL>{});
  };
  for (int t = 0; t < ntiles; t += 2) {
    tile(std::integral_constant<int, 0>{}, t);
    advance(std::integral_constant<int, 0>{}, t);
    if (t + 1 < ntiles) {
      tile(std::integral_constant<int, 1>{}, t + 1);
      advance(std::integral_constant<int, 1>{}, t + 1);
    }
  }
  stamp(3);
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
  if constexpr (STAMP) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    stamp(4);
    if (tid == 0) a.stamps[blockIdx.x * 8 + 5] = (unsigned long long)ntiles;
  }
}

// ---------------------------------------------------------------------------------------------
// dK / dV, persistent (round 3).  A timeline of fa_bwd_dkv_pipe_kernel (s_memrealtime stamps,
// tools/dkv_timeline.py, profiles/attn_dkv_r3.txt) at B12 S2048 H32: per workgroup 4.9 us of
// prologue (K / V + first tile), 4.6 us of epilogue and a 6.1 us gap before the CU's next
// workgroup starts, against 2.2 us per 64-row tile and 17 tiles per workgroup on average: ~30 %
// of the kernel outside the tile loop.  Here one workgroup per CU stays resident and takes
// (batch * kv-head, key-block) items from a per-XCD work queue (one atomic per item; queue x =
// blockIdx % 8 holds its heads' items head-major, heaviest key block first, so the ~32 concurrent
// items of an XCD share two or three heads' Q / dO in its L2 while the dynamic order balances the
// causal costs).  The Q / dO DMA stream runs on across items (the next item's first tiles land
// under the current item's last ones), the next item's K / V fragments load under the last tile's
// products, and the barrier sits before the second-half dV / dK MFMAs so the next tile's first
// fragment reads land under them.  Scope: causal, head_dim 128, S % 128 == 0, no packed documents
// (every item then has >= 2 tiles, which bounds the issue cursor's lead to two items).
// wq: int32[8] per-XCD item counters, zeroed by the host before every launch.
template <bool STAMP>
__global__ __launch_bounds__(256, 1) void fa_bwd_dkv_persist_kernel(BwdArgs a, int* __restrict__ wq) {
  constexpr int HD = 128;
  constexpr int NKS = HD / 16;
  constexpr int NDB = HD / 32;
  constexpr int ROWB = HD * 2;
  constexpr int TILE_B = KV_QT * ROWB;
  constexpr int NP = TILE_B / 1024 / 4;
  constexpr int RC_B = KV_QT * 4;
  constexpr int BUF_B = 2 * TILE_B + 4 * RC_B;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * BUF_B + 64];  // + item ids
  // item ids handed from thread 0 to the workgroup: [1] [2] the first two items; [3 + (k & 1)] the
  // lookahead popped at the k-th cursor switch (written after a barrier, read after the next one).
  // Two slots: with 2-tile items (the last key block of a head, one q-head per kv-head) a switch
  // can follow the previous one right after the barrier at which that one's lookahead is read —
  // one slot let thread 0 overwrite it before the slower waves had read it (waves then disagreed
  // on the next item)
  int* item_w = reinterpret_cast<int*>(smem + 2 * BUF_B);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const int nkb = a.S / KV_KB;
  const int BH = a.B * a.Hkv;
  const bool per_xcd = BH % 8 == 0;
  const int xq = per_xcd ? (int)(blockIdx.x & 7) : 0;
  const int n_items = (per_xcd ? BH / 8 : BH) * nkb;
  const int bh_base = per_xcd ? xq * (BH / 8) : 0;
  const int group = a.Hq / a.Hkv;
  auto pop = [&]() __attribute__((always_inline)) -> int {  // thread 0
    const int j = __hip_atomic_fetch_add(wq + xq, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return j < n_items ? j : -1;
  };
  if (tid == 0) {
    const int i0 = pop();
    item_w[1] = i0;
    item_w[2] = i0 >= 0 ? pop() : -1;
  }
  __syncthreads();
  int cur = __builtin_amdgcn_readfirstlane(item_w[1]);
  int nxt = __builtin_amdgcn_readfirstlane(item_w[2]);
  if (cur < 0) return;

  const unsigned lds0 = lds_addr(smem);
  unsigned vq[NP], vd[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int byte = (i * 4 + wave) * 1024 + lane * 16;
    const int row = byte / ROWB;
    const int lch = ((byte % ROWB) >> 4) ^ swz_tr<HD>(row);
    vq[i] = (unsigned)((row * a.q_ss + lch * 8) * 2);
    vd[i] = (unsigned)((row * a.do_ss + lch * 8) * 2);
  }
  const float* rc_src = a.rck_w + (wave == 1 ? a.rc_n : 0);
  const unsigned rc_off =
      (unsigned)((32 * (lane >> 5) + 8 * ((lane >> 2) & 3) + 4 * ((lane >> 4) & 1) + (lane & 3)) * 4);

  // ---- issue cursor: the Q / dO / row-constant DMA stream over (item, q-head of the GQA group, tile)
  int iss = cur, iq0 = 0, iq_start = 0, ig = 0;
  const unsigned short *qh = nullptr, *dh = nullptr;
  const float* rh = nullptr;
  bool look_pending = false;
  int n_switch = 0;  // cursor switches so far (wave-uniform)
  // items the cursor entered (or -1: the stream ended) that compute has not started, in order: the
  // cursor switches when it issues an item's LAST tile, so with a 2-tile next item it can switch
  // twice during one compute item (one variable lost the first of the two: a skipped item)
  int pend0 = -1, pend1 = -1, npend = 0;
  auto iss_begin = [&](int item) __attribute__((always_inline)) {
    const int bh = bh_base + item / nkb, kb = item % nkb;
    const int bb = bh / a.Hkv, hkk = bh % a.Hkv;
    iq_start = kb * KV_KB;
    iq0 = iq_start;
    ig = 0;
    qh = a.q + bb * a.q_sb + (long)(hkk * group) * a.q_sh;
    dh = a.dout + bb * a.do_sb + (long)(hkk * group) * a.do_sh;
    rh = rc_src + ((long)bb * a.Hq + hkk * group) * a.S;
  };
  iss_begin(cur);
  auto issue = [&](auto slot_c) __attribute__((always_inline)) {
    constexpr int SLC = decltype(slot_c)::value;
    i32x4_t rq = buf_rsrc(qh + (long)iq0 * a.q_ss, (unsigned)(((KV_QT - 1) * a.q_ss + HD) * 2));
    i32x4_t rd = buf_rsrc(dh + (long)iq0 * a.do_ss, (unsigned)(((KV_QT - 1) * a.do_ss + HD) * 2));
    i32x4_t rr = buf_rsrc(rh + iq0, (unsigned)(KV_QT * 4));
    asm volatile("s_nop 4" : "+s"(rq), "+s"(rd), "+s"(rr));
    const unsigned slot = lds0 + (unsigned)(SLC * BUF_B);
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      buf_dma16(rq, vq[i], slot + (i * 4 + wave) * 1024);
      buf_dma16(rd, vd[i], slot + TILE_B + (i * 4 + wave) * 1024);
    }
    buf_dma4(rr, rc_off, slot + 2 * TILE_B + wave * RC_B);
    iq0 += KV_QT;
    if (iq0 >= a.S) {
      if (++ig < group) {  // next q-head of the GQA group
        iq0 = iq_start;
        qh += a.q_sh;
        dh += a.do_sh;
        rh += a.S;
      } else {  // next item: it becomes the compute side's next item, thread 0 pops a lookahead
        iss = nxt;
        if (iss >= 0) {
          iss_begin(iss);
          if (tid == 0) item_w[3 + (n_switch & 1)] = pop();
          look_pending = true;
          ++n_switch;
        }
        if (npend == 0) pend0 = iss;
        else pend1 = iss;
        ++npend;
      }
    }
  };

  bf16x8_t kf[NKS], vf[NKS];
  auto load_kv = [&](int item) __attribute__((always_inline)) {
    const int bh = bh_base + item / nkb, kb = item % nkb;
    const int bb = bh / a.Hkv, hkk = bh % a.Hkv;
    const int key = kb * KV_KB + wave * 32 + r;
    const unsigned short* Kp = a.k + bb * a.k_sb + hkk * a.k_sh + (long)key * a.k_ss + 8 * hh;
    const unsigned short* Vp = a.v + bb * a.v_sb + hkk * a.v_sh + (long)key * a.v_ss + 8 * hh;
    // "+a": the new fragments overwrite the old ones in place (no second register set)
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      asm volatile("global_load_dwordx4 %0, %1, off" : "+a"(kf[ks]) : "v"(Kp + 16 * ks) : "memory");
      asm volatile("global_load_dwordx4 %0, %1, off" : "+a"(vf[ks]) : "v"(Vp + 16 * ks) : "memory");
    }
  };

  // prologue: tile 0's DMA with the K / V fragments under it, one wait, then tile 1's DMA
  issue(std::integral_constant<int, 0>{});
  load_kv(cur);
  asm volatile("s_waitcnt vmcnt(0)"
               : "+a"(kf[0]), "+a"(kf[1]), "+a"(kf[2]), "+a"(kf[3]), "+a"(kf[4]), "+a"(kf[5]), "+a"(kf[6]),
                 "+a"(kf[7]), "+a"(vf[0]), "+a"(vf[1]), "+a"(vf[2]), "+a"(vf[3]), "+a"(vf[4]), "+a"(vf[5]),
                 "+a"(vf[6]), "+a"(vf[7])
               :
               : "memory");
  __builtin_amdgcn_s_barrier();
  issue(std::integral_constant<int, 1>{});
  f32x16 dk[NDB], dv[NDB];
#pragma unroll
  for (int d = 0; d < NDB; ++d) {
    const bf16x8_t z = {};
    asm volatile("s_nop 2\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %1, 0" : "=a"(dk[d]) : "v"(z));  // see acc_zero
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %1, 0" : "=a"(dv[d]) : "v"(z));
  }
  const float c = a.scale_log2;

  int n_done = 0;  // STAMP: items finished by this workgroup
  auto stamp = [&](int k) __attribute__((always_inline)) {
    if constexpr (STAMP) {
      if (tid == 0 && n_done < 64)
        a.stamps[(blockIdx.x * 64 + n_done) * 4 + k] = k == 3 ? (unsigned long long)cur : __builtin_amdgcn_s_memrealtime();
    }
  };
  for (;;) {  // ---- items
    stamp(0);
    stamp(3);
    const int bh = bh_base + cur / nkb, kb = cur % nkb;
    const int b = bh / a.Hkv, hk = bh % a.Hkv;
    const int k0 = kb * KV_KB;
    const int wkey0 = k0 + wave * 32;
    const int my_key = wkey0 + r;
    const int ntiles = group * ((a.S - k0) / KV_QT);  // even
    int q0 = k0;
    auto apply_mask = [&](f32x16& s, int h) __attribute__((always_inline)) {
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int row0 = q0 + 32 * h + 8 * gq + 4 * hh;
#pragma unroll
        for (int j = 0; j < 4; ++j) s[4 * gq + j] = my_key <= row0 + j ? s[4 * gq + j] : -INFINITY;
      }
    };
    // one tile in ring slot SL (as fa_bwd_dkv_pipe_kernel)
    auto tile = [&](auto slot_c) __attribute__((always_inline)) {
      constexpr int SL = decltype(slot_c)::value;
      const bool live = !(wkey0 > q0 + KV_QT - 1);
      if (!live) return;
      const unsigned char* Qs = smem + SL * BUF_B;
      const unsigned char* Ds = Qs + TILE_B;
      const float* lse_s = reinterpret_cast<const float*>(Ds + TILE_B);
      const float* del_s = lse_s + KV_QT;
      const bool need_mask = wkey0 + 31 > q0;
      f32x16 s0 = *reinterpret_cast<const f32x16*>(lse_s + 16 * hh);
      f32x16 p0 = *reinterpret_cast<const f32x16*>(del_s + 16 * hh);
      bf16x8_t qa[NKS], da[NKS];
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        qa[ks] = lds_read_b128(Qs, tr_off<HD>(r, 2 * ks + hh));
        da[ks] = lds_read_b128(Ds, tr_off<HD>(r, 2 * ks + hh));
      }
      f32x16 s1 = *reinterpret_cast<const f32x16*>(lse_s + 32 + 16 * hh);
      f32x16 p1 = *reinterpret_cast<const f32x16*>(del_s + 32 + 16 * hh);
      bf16x8_t qb[NKS], db[NKS];
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {  // S0 / dP0 with the second half's fragment reads
        mfma_v(s0, qa[ks], kf[ks]);
        qb[ks] = lds_read_b128(Qs, tr_off<HD>(32 + r, 2 * ks + hh));
        mfma_v(p0, da[ks], vf[ks]);
        db[ks] = lds_read_b128(Ds, tr_off<HD>(32 + r, 2 * ks + hh));
      }
      if (need_mask) apply_mask(s0, 0);
      unsigned pw0[8], dw0[8];
      bf16x8_t td[2][NDB], tq[2][NDB];
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {  // X: S1 / dP1 || softmax(half 0), T0 reads
        x_step(s1, p1, qb[ks], kf[ks], db[ks], vf[ks], s0[2 * ks], s0[2 * ks + 1], p0[2 * ks], p0[2 * ks + 1], c,
               pw0[ks], dw0[ks]);
        const int st = ks >> 2, d = ks & 3;
        td[st][d] = tr_frag<HD>(Ds, 16 * st, d * 32, lane);
        tq[st][d] = tr_frag<HD>(Qs, 16 * st, d * 32, lane);
      }
      if (need_mask) apply_mask(s1, 1);
      unsigned pw1[8], dw1[8];
      bf16x8_t cd[2][NDB], cq[2][NDB];
#pragma unroll
      for (int st = 0; st < 2; ++st) {  // Y: dV / dK(half 0) || softmax(half 1), T1 reads
        const bf16x8_t pb = words8(pw0[4 * st], pw0[4 * st + 1], pw0[4 * st + 2], pw0[4 * st + 3]);
        const bf16x8_t sb = words8(dw0[4 * st], dw0[4 * st + 1], dw0[4 * st + 2], dw0[4 * st + 3]);
#pragma unroll
        for (int d = 0; d < NDB; ++d) {
          const int i = 4 * st + d;
          y_step(dv[d], dk[d], td[st][d], tq[st][d], pb, sb, s1[2 * i], s1[2 * i + 1], p1[2 * i], p1[2 * i + 1], c,
                 pw1[i], dw1[i]);
          cd[st][d] = tr_frag<HD>(Ds, 32 + 16 * st, d * 32, lane);
          cq[st][d] = tr_frag<HD>(Qs, 32 + 16 * st, d * 32, lane);
        }
      }
#pragma unroll
      for (int st = 0; st < 2; ++st) {  // dV / dK (half 1)
        const bf16x8_t pb = words8(pw1[4 * st], pw1[4 * st + 1], pw1[4 * st + 2], pw1[4 * st + 3]);
        const bf16x8_t sb = words8(dw1[4 * st], dw1[4 * st + 1], dw1[4 * st + 2], dw1[4 * st + 3]);
#pragma unroll
        for (int d = 0; d < NDB; ++d) z_step(dv[d], dk[d], cd[st][d], cq[st][d], pb, sb);
      }
    };
    // after each tile: reads of its slot retired, the next tile's DMA landed -> barrier; the slot
    // takes the stream's tile two ahead (maybe the next item's)
    auto advance = [&](auto slot_c) __attribute__((always_inline)) {
      constexpr int SL = decltype(slot_c)::value;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      vm_wait_n<0>();
      __builtin_amdgcn_s_barrier();
      if (look_pending) {
        nxt = __builtin_amdgcn_readfirstlane(item_w[3 + ((n_switch - 1) & 1)]);
        look_pending = false;
      }
      if (iss >= 0) issue(std::integral_constant<int, SL>{});
      q0 += KV_QT;
      if (q0 >= a.S) q0 = k0;  // next q-head of the GQA group
    };
    for (int t = 0; t < ntiles; t += 2) {
      tile(std::integral_constant<int, 0>{});
      advance(std::integral_constant<int, 0>{});
      tile(std::integral_constant<int, 1>{});
      advance(std::integral_constant<int, 1>{});
    }
    stamp(1);
    // ---- item end: dK (scaled, with the RoPE backward fused) and dV stored, then the next item's
    //      K / V fragments loaded behind the stores and retired by one wait.  The RoPE tables are
    //      plain loads (see below); the K / V loads come after their last use, so the compiler's
    //      own wait for the tables never covers them.
    {
      const long tok = (long)b * a.S + my_key;
      unsigned short* dkp = a.dk + tok * a.dk_st + (long)hk * HD;
      unsigned short* dvp = a.dv + tok * a.dv_st + (long)hk * HD;
      const bool rope = a.cos_t != nullptr;
      f32x4 cs[NDB / 2][4], sn[NDB / 2][4];
      if (rope) {
        const long p = a.rope_pos ? (long)a.rope_pos[tok] : tok % a.rope_S;
        const float* cr = a.cos_t + p * (HD / 2);
        const float* sr = a.sin_t + p * (HD / 2);
#pragma unroll
        for (int d = 0; d < NDB / 2; ++d)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int col = d * 32 + 8 * g + 4 * hh;
            // plain loads: the compiler tracks them (its waits are conservative around the asm
            // ops).  As inline-asm loads, hipcc copied the "=v" destinations into other registers
            // right after issue and reused them for the next addresses while the data was still
            // in flight — the landing data corrupted a later load's address (illegal access)
            cs[d][g] = *reinterpret_cast<const f32x4*>(cr + col);
            sn[d][g] = *reinterpret_cast<const f32x4*>(sr + col);
          }
      }
      // the last MFMAs' results -> the AGPR reads below: 8-pass XDL write, 12+ wait states; the "+a"
      // operands order every read after the padding
#pragma unroll
      for (int d = 0; d < NDB; ++d) asm volatile("s_nop 7\n\ts_nop 7" : "+a"(dk[d]), "+a"(dv[d]));
      auto st8 = [&](unsigned short* p, const float* x, float mul) __attribute__((always_inline)) {
        s2_t w;
        w[0] = (unsigned)f2bf(x[0] * mul) | ((unsigned)f2bf(x[1] * mul) << 16);
        w[1] = (unsigned)f2bf(x[2] * mul) | ((unsigned)f2bf(x[3] * mul) << 16);
        asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(p), "v"(w) : "memory");
      };
#pragma unroll
      for (int d = 0; d < NDB / 2; ++d) {
        const f32x16 x1 = acc_copy(dk[d]), x2 = acc_copy(dk[d + NDB / 2]);
        acc_zero(dk[d]);
        acc_zero(dk[d + NDB / 2]);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int col = d * 32 + 8 * g + 4 * hh;  // < HD / 2
          float lo[4], hi[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float c1 = rope ? cs[d][g][j] : 1.f, s1 = rope ? sn[d][g][j] : 0.f;
            lo[j] = x1[4 * g + j] * c1 + x2[4 * g + j] * s1;
            hi[j] = x2[4 * g + j] * c1 - x1[4 * g + j] * s1;
          }
          st8(dkp + col, lo, a.scale);
          st8(dkp + col + HD / 2, hi, a.scale);
        }
      }
#pragma unroll
      for (int d = 0; d < NDB; ++d) {
        const f32x16 x = acc_copy(dv[d]);
        acc_zero(dv[d]);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          float y[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) y[j] = x[4 * g + j];
          st8(dvp + d * 32 + 8 * g + 4 * hh, y, 1.f);
        }
      }
      load_kv(pend0 >= 0 ? pend0 : cur);  // one code path (no next item: a harmless re-load)
      // the K / V loads retire here: the fragments are operands of this statement, so hipcc cannot
      // place a register copy of them (e.g. to coalesce the item loop's back edge) before the data
      // has landed — without them a v_accvgpr_mov could read the in-flight destination
      asm volatile("s_waitcnt vmcnt(0)"
                   : "+a"(kf[0]), "+a"(kf[1]), "+a"(kf[2]), "+a"(kf[3]), "+a"(kf[4]), "+a"(kf[5]), "+a"(kf[6]),
                     "+a"(kf[7]), "+a"(vf[0]), "+a"(vf[1]), "+a"(vf[2]), "+a"(vf[3]), "+a"(vf[4]), "+a"(vf[5]),
                     "+a"(vf[6]), "+a"(vf[7])
                   :
                   : "memory");
    }
    stamp(2);
    ++n_done;
    if (pend0 < 0) break;  // the stream ended with this item
    cur = pend0;
    pend0 = pend1;
    pend1 = -1;
    --npend;
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
  // K^T fragment offsets per 32-column d block (tr_frag_at; the rows kb * 32 + 16 st are multiples
  // of 16): no per-read address arithmetic in the tile loop
  int klo[NDB], khi[NDB];
#pragma unroll
  for (int d = 0; d < NDB; ++d) tr_frag_offs<HD>(d * 32, lane, klo[d], khi[d]);
  // K (tr image) / V (row image) row-fragment offsets per k-step: both swizzles of rows kb * 32 + r
  // depend on r only, so kb folds into the ds_read immediate
  int kro[NKS], vro[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    kro[ks] = tr_off<HD>(r, 2 * ks + hh);
    vro[ks] = row_off<HD>(r, 2 * ks + hh);
  }

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
        s = mfma32(lds_read_b128(Ks, kb * 32 * (HD * 2) + kro[ks]), qf[ks], s);
        dp = mfma32(lds_read_b128(Vs, kb * 32 * (HD * 2) + vro[ks]), df[ks], dp);
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
        for (int d = 0; d < NDB; ++d) dq[d] = mfma32(tr_frag_at<HD>(Ks, kb * 32 + 16 * st, klo[d], khi[d]), sbf, dq[d]);
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

// dK/dV kernel (A/B knob dkv): 0 = unpipelined, 1 = software-pipelined, 2 (default) =
// persistent where it applies (causal, head_dim 128, S % 128, no documents), else pipelined.
// B12 S2048 H32 D128 (tools/attn_ablate.py): 1.24 / 1.12 / 0.98-1.00 ms
int dkv_mode() {
  const int64_t m = knob("dkv", 2);
  return (m >= 0 && m <= 2) ? (int)m : 2;
}

// the persistent dK/dV kernel's per-XCD item counters: one buffer per (device, stream), zeroed
// before every launch on that stream.  Launches on one stream are ordered, so they may share a
// buffer; two streams (or threads launching on them) never do.  The map is mutex-guarded.
int* dkv_queue(hipStream_t s) {
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, int*> bufs;
  int dev = 0;
  LLMCTL_HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(mu);
  int*& q = bufs[{dev, s}];
  if (q == nullptr) LLMCTL_HIP_CHECK(hipMalloc(&q, 64 * sizeof(int)));
  return q;
}

// dkv_impl: -1 = default (knob dkv), 0 = unpipelined kernel, 1 = pipelined where built
template <int HD, bool CAUSAL, bool DOC>
void launch_bwd(const BwdArgs& a, hipStream_t s, bool do_dq, bool do_dkv, int dkv_impl) {
  if (do_dq) {
    const int nqb = (a.S + DQ_QB - 1) / DQ_QB;
    hipLaunchKernelGGL((fa_bwd_dq_kernel<HD, CAUSAL, DOC>), dim3((unsigned)(a.B * a.Hq * nqb)), dim3(256), 0, s, a);
  }
  if (do_dkv) {
    const int nkb = (a.S + KV_KB - 1) / KV_KB;
    const dim3 grid((unsigned)(a.B * a.Hkv * nkb));
    if constexpr (HD == 128 && CAUSAL) {  // the full-attention build spills (not the training path)
      if (dkv_impl == 2 && a.stamps != nullptr) {
        hipLaunchKernelGGL((fa_bwd_dkv_pipe_kernel<HD, CAUSAL, DOC, true>), grid, dim3(256), 0, s, a);
        return;
      }
      if constexpr (!DOC) {  // persistent form: S % 128 (>= 2 tiles per item)
        if (a.S % KV_KB == 0 && (dkv_impl == 3 || dkv_impl == 4 || (dkv_impl < 0 && dkv_mode() == 2))) {
          int* wq = dkv_queue(s);
          LLMCTL_HIP_CHECK(hipMemsetAsync(wq, 0, 8 * sizeof(int), s));
          int nwg = std::min<long>((long)num_cus(), (long)a.B * a.Hkv * nkb);
          // per-XCD queues (B*Hkv % 8 == 0) are drained by blocks with blockIdx & 7 == queue:
          // fewer than 8 workgroups would leave queues without a consumer
          const int min_wg = ((long)a.B * a.Hkv) % 8 == 0 ? 8 : 1;
          if (const int64_t e = knob("dkv_nwg", 0); e > 0) nwg = std::max<int>(min_wg, std::min<int>(nwg, (int)e));  // debug
          nwg = std::max(nwg, min_wg);
          if (a.stamps != nullptr)
            hipLaunchKernelGGL(fa_bwd_dkv_persist_kernel<true>, dim3((unsigned)nwg), dim3(256), 0, s, a, wq);
          else
            hipLaunchKernelGGL(fa_bwd_dkv_persist_kernel<false>, dim3((unsigned)nwg), dim3(256), 0, s, a, wq);
          return;
        }
      }
      if (dkv_impl == 1 || dkv_impl == 3 || (dkv_impl < 0 && dkv_mode() >= 1)) {
        hipLaunchKernelGGL((fa_bwd_dkv_pipe_kernel<HD, CAUSAL, DOC>), grid, dim3(256), 0, s, a);
        return;
      }
    }
    hipLaunchKernelGGL((fa_bwd_dkv_kernel<HD, CAUSAL, DOC>), grid, dim3(256), 0, s, a);
  }
}

void dispatch_bwd(const BwdArgs& a, int D, bool causal, bool doc, hipStream_t s, bool do_dq = true,
                  bool do_dkv = true, int dkv_impl = -1) {
  if (doc) {
    if (D == 128) launch_bwd<128, true, true>(a, s, do_dq, do_dkv, dkv_impl);
    else launch_bwd<64, true, true>(a, s, do_dq, do_dkv, dkv_impl);
  } else if (D == 128) {
    if (causal) launch_bwd<128, true, false>(a, s, do_dq, do_dkv, dkv_impl);
    else launch_bwd<128, false, false>(a, s, do_dq, do_dkv, dkv_impl);
  } else {
    if (causal) launch_bwd<64, true, false>(a, s, do_dq, do_dkv, dkv_impl);
    else launch_bwd<64, false, false>(a, s, do_dq, do_dkv, dkv_impl);
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

// timing / A-B entry for tools/attn_ablate.py and the GPU tests (causal, no documents): abl 0 = both
// kernels, 1 = dK/dV kernel only (its row constants prepared by two small torch ops), 2 = dQ kernel
// only, 3 / 4 = dK/dV only through the unpipelined / pipelined kernel, 5 = the pipelined kernel's
// diagnostic timeline build: 8 u64 per workgroup written over dq's storage (see the kernel's STAMP),
// 6 = dK/dV only through the persistent kernel, 7 = its timeline build (4 u64 per item, 64 items per
// workgroup, over dq's storage).
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
  if (abl == 5 || abl == 7) {
    LLMCTL_CHECK(dq.numel() * 2 >= (long)q.size(0) * k.size(2) * ((q.size(1) + KV_KB - 1) / KV_KB) * 64,
                 "fa_bwd_ablate: dq too small for the timeline");
    a.stamps = reinterpret_cast<unsigned long long*>(dq.data_ptr());
  }
  auto rck = row_consts(a, lse);
  if (abl == 1 || abl >= 3) {  // no dQ kernel to write them
    rck.narrow(0, 0, lse.numel()).copy_(lse.reshape(-1) * (-1.0 / scale));
    rck.narrow(0, lse.numel(), lse.numel()).copy_(-delta.reshape(-1));
  }
  dispatch_bwd(a, D, true, false, stream(), abl == 0 || abl == 2, abl != 2, abl >= 3 ? (int)abl - 3 : -1);
}

TORCH_LIBRARY_IMPL(llmctl, CUDA, m) {
  m.impl("flash_attn_bwd", &flash_attn_bwd);
  m.impl("flash_attn_bwd_qkv", &flash_attn_bwd_qkv);
  m.impl("fa_bwd_ablate", &fa_bwd_ablate);
}

}  // namespace llmctl
