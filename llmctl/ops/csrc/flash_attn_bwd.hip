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
//   rows of one (batch, q-head), Q and dO fragments in registers, K/V tiles of 64 keys staged
//   through LDS (register staging split around the MFMAs, guide T14); "swapped" products keep the
//   key on the registers so dS^T is directly the B operand of dQ^T += K^T dS^T.  dQ is written
//   once, in bf16.
// A pre-kernel computes delta.
#include "attn_common.h"

namespace llmctl {
using namespace attn;
namespace {

constexpr float LOG2E = 1.4426950408889634f;
constexpr int KV_KB = 128;  // keys per dK/dV workgroup
constexpr int KV_QT = 64;   // query rows per streamed tile
constexpr int KV_NBUF = 3;  // LDS ring depth
constexpr int DQ_QB = 128;  // query rows per dQ workgroup
constexpr int DQ_KB = 64;   // keys per dQ tile
constexpr int DKV_VAR = 0;  // dK/dV loop-body schedule (see fa_bwd_dkv_kernel); A/B: fa_bwd_ablate 3/4

struct BwdArgs {
  const unsigned short *q, *k, *v, *dout;
  const float* lse;    // [B,Hq,S] natural log
  const float* delta;  // [B,Hq,S]
  unsigned short *dq, *dk, *dv;  // [B,S,H,HD] contiguous
  int B, S, Hq, Hkv;
  long q_sb, q_ss, q_sh, k_sb, k_ss, k_sh, v_sb, v_ss, v_sh, do_sb, do_ss, do_sh;
  float scale, scale_log2;
  const int* doc;  // [B, S] document start per token (packed sequences), or nullptr
};

template <int HD>
__global__ __launch_bounds__(256) void delta_kernel(const unsigned short* __restrict__ dout,
                                                     const unsigned short* __restrict__ o, float* __restrict__ delta,
                                                     int B, int S, int Hq, long do_sb, long do_ss, long do_sh,
                                                     long o_sb, long o_ss, long o_sh) {
  constexpr int LPR = HD / 8;  // lanes per row
  const long gid = (long)blockIdx.x * 256 + threadIdx.x;
  const long row = gid / LPR;
  const int sub = gid % LPR;
  const long R = (long)B * S * Hq;
  float s = 0.f;
  int b = 0, hq = 0, sq = 0;
  if (row < R) {
    b = row / ((long)S * Hq);
    const long rem = row % ((long)S * Hq);
    sq = rem / Hq;
    hq = rem % Hq;
    float x[8], y[8];
    load8(dout + b * do_sb + sq * do_ss + hq * do_sh + sub * 8, x);
    load8(o + b * o_sb + sq * o_ss + hq * o_sh + sub * 8, y);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += x[j] * y[j];
  }
#pragma unroll
  for (int off = LPR / 2; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if (row < R && sub == 0) delta[((long)b * Hq + hq) * S + sq] = s;
}

__device__ __forceinline__ void store_bf16x4(unsigned short* p, const float* x, float mul) {
  unsigned short w[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) w[j] = f2bf(x[j] * mul);
  *reinterpret_cast<uint2*>(p) =
      make_uint2((unsigned)w[0] | ((unsigned)w[1] << 16), (unsigned)w[2] | ((unsigned)w[3] << 16));
}

// =============================================================================================
// dK / dV
// =============================================================================================
template <int HD, bool CAUSAL, bool DOC, int VAR = DKV_VAR>
__global__ __launch_bounds__(256, 1) void fa_bwd_dkv_kernel(BwdArgs a) {
  constexpr int NKS = HD / 16;
  constexpr int NDB = HD / 32;
  constexpr int ROWB = HD * 2;
  constexpr int TILE_B = KV_QT * ROWB;     // one Q (or dO) tile
  constexpr int NP = TILE_B / 1024 / 4;    // 1-KiB DMA pieces per wave per operand
  constexpr int VM = 2 * NP + 1;           // DMA instructions per wave per tile
  constexpr int RC_B = KV_QT * 4;          // one row-constant vector
  constexpr int BUF_B = 2 * TILE_B + 4 * RC_B;  // Q | dO | lse | delta | doc | (dummy)
  __shared__ __attribute__((aligned(1024))) unsigned char smem[KV_NBUF * BUF_B];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const int BH = a.B * a.Hkv;
  const int bh = blockIdx.x % BH;
  const int kblk = blockIdx.x / BH;  // small kblk = most query tiles under causal: dispatched first
  const int b = bh / a.Hkv, hk = bh % a.Hkv;
  const int group = a.Hq / a.Hkv;
  const int k0 = kblk * KV_KB;
  const int wkey0 = k0 + wave * 32;
  const int my_key = wkey0 + r;

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
    q_end = lo;
  }
  const int nq = q_end > q_start ? (q_end - q_start + KV_QT - 1) / KV_QT : 0;
  const int ntiles = group * nq;
  const unsigned lds0 = lds_addr(smem);

  // ---- DMA of tile t into ring slot t % 3: every wave issues exactly VM instructions
  auto issue = [&](int t) {
    const int g = t / nq;
    const int q0 = q_start + (t - g * nq) * KV_QT;
    const int hq = hk * group + g;
    const unsigned slot = lds0 + (unsigned)((t % KV_NBUF) * BUF_B);
    const unsigned short* Qp = a.q + b * a.q_sb + hq * a.q_sh;
    const unsigned short* Dp = a.dout + b * a.do_sb + hq * a.do_sh;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int piece = i * 4 + wave;
      const int byte = piece * 1024 + lane * 16;
      const int row = byte / ROWB;
      const int pch = (byte % ROWB) >> 4;                // physical chunk in the tr image
      const int lch = pch ^ swz_tr<HD>(row);             // logical chunk it holds
      const long qq = min(q0 + row, a.S - 1);            // rows past S: P masked to 0
      dma16(Qp + qq * a.q_ss + lch * 8, slot + piece * 1024);
      dma16(Dp + qq * a.do_ss + lch * 8, slot + TILE_B + piece * 1024);
    }
    const int qq = min(q0 + lane, a.S - 1);
    const long rc = ((long)b * a.Hq + hq) * a.S + qq;
    const void* src = wave == 1 ? (const void*)(a.delta + rc)
                    : (DOC && wave == 2) ? (const void*)(a.doc + (long)b * a.S + qq)
                                         : (const void*)(a.lse + rc);
    dma4(src, slot + 2 * TILE_B + wave * RC_B);
  };

  if (ntiles > 0) issue(0);
  if (ntiles > 1) issue(1);
  for (int t = 0; t < ntiles; ++t) {
    if (t + 1 < ntiles) vm_wait<VM>();  // this wave's DMA of tile t landed (t+1 stays in flight)
    else vm_wait<0>();
    __builtin_amdgcn_s_barrier();       // ... and every other wave's; slot (t+2)%3 is free
    if (t + 2 < ntiles) issue(t + 2);

    const int g = t / nq;
    const int q0 = q_start + (t - g * nq) * KV_QT;
    const unsigned char* Qs = smem + (t % KV_NBUF) * BUF_B;
    const unsigned char* Ds = Qs + TILE_B;
    const float* lse_s = reinterpret_cast<const float*>(Ds + TILE_B);
    const float* del_s = lse_s + KV_QT;
    const int* doc_s = reinterpret_cast<const int*>(del_s + KV_QT);
    // no early-out for tiles a wave sees nothing of (only the first tile of a causal block, for
    // half the waves): a branch here makes hipcc shuttle dK/dV between AGPRs and VGPRs every tile

    // ---- per 32-row half h: S = Q K^T, dP = dO V^T (q on regs, key on lane), then
    //      dV^T += dO^T P and dK^T += Q^T dS (sum over the half's rows = the registers).
    //      Masks are branch-free selects.  VAR 0: half after half; VAR 1: both halves'
    //      S/dP chains first (the second half's MFMAs cover the first half's exp/VALU work);
    //      VAR 2: as 1 with each half's operand fragments read into registers ahead of its MFMAs.
    auto sdp = [&](int h, f32x16& s, f32x16& dp) {
#pragma unroll
      for (int i = 0; i < 16; ++i) s[i] = dp[i] = 0.f;
      if constexpr (VAR == 2) {
        bf16x8_t qa[NKS], da[NKS];
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          qa[ks] = lds_read_b128(Qs, tr_off<HD>(32 * h + r, 2 * ks + hh));
          da[ks] = lds_read_b128(Ds, tr_off<HD>(32 * h + r, 2 * ks + hh));
        }
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          s = mfma32(qa[ks], kf[ks], s);
          dp = mfma32(da[ks], vf[ks], dp);
        }
      } else {
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          const bf16x8_t qa = lds_read_b128(Qs, tr_off<HD>(32 * h + r, 2 * ks + hh));
          const bf16x8_t da = lds_read_b128(Ds, tr_off<HD>(32 * h + r, 2 * ks + hh));
          s = mfma32(qa, kf[ks], s);
          dp = mfma32(da, vf[ks], dp);
        }
      }
    };
    auto soft = [&](int h, const f32x16& s, const f32x16& dp, bf16x8_t* pb, bf16x8_t* sb) {
      float p[16], dsv[16];
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int row0 = 32 * h + 8 * gq + 4 * hh;  // rows of registers 4gq .. 4gq+3
        const float4 l4 = *reinterpret_cast<const float4*>(lse_s + row0);
        const float4 d4 = *reinterpret_cast<const float4*>(del_s + row0);
        int4 s4 = make_int4(0, 0, 0, 0);
        if constexpr (DOC) s4 = *reinterpret_cast<const int4*>(doc_s + row0);
        const float lv[4] = {l4.x, l4.y, l4.z, l4.w};
        const float dv4[4] = {d4.x, d4.y, d4.z, d4.w};
        const int sv[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int i = 4 * gq + j;
          const int qq = q0 + row0 + j;
          bool dead = (qq >= a.S) | (my_key >= a.S);
          if constexpr (CAUSAL) dead |= my_key > qq;
          if constexpr (DOC) dead |= my_key < sv[j];
          const float pv = dead ? 0.f : fast_exp2(s[i] * a.scale_log2 - lv[j] * LOG2E);
          p[i] = pv;
          dsv[i] = pv * (dp[i] - dv4[j]);
        }
      }
      pb[0] = to_bf16x8(p);
      pb[1] = to_bf16x8(p + 8);
      sb[0] = to_bf16x8(dsv);
      sb[1] = to_bf16x8(dsv + 8);
    };
    auto dvdk = [&](int h, const bf16x8_t* pb, const bf16x8_t* sb) {
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int d = 0; d < NDB; ++d) {
          const bf16x8_t da = tr_frag<HD>(Ds, 32 * h + 16 * st, d * 32, lane);
          dv[d] = mfma32(da, pb[st], dv[d]);
          const bf16x8_t qa = tr_frag<HD>(Qs, 32 * h + 16 * st, d * 32, lane);
          dk[d] = mfma32(qa, sb[st], dk[d]);
        }
    };
    if constexpr (VAR == 0) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        f32x16 s, dp;
        bf16x8_t pb[2], sb[2];
        sdp(h, s, dp);
        soft(h, s, dp, pb, sb);
        dvdk(h, pb, sb);
      }
    } else {
      f32x16 s0, dp0, s1, dp1;
      bf16x8_t pb0[2], sb0[2], pb1[2], sb1[2];
      sdp(0, s0, dp0);
      sdp(1, s1, dp1);
      soft(0, s0, dp0, pb0, sb0);
      dvdk(0, pb0, sb0);
      soft(1, s1, dp1, pb1, sb1);
      dvdk(1, pb1, sb1);
    }
  }
  // ---- write dK (scaled), dV: lane = key, registers = d
  if (my_key < a.S) {
    unsigned short* dkp = a.dk + ((long)b * a.S + my_key) * a.Hkv * HD + (long)hk * HD;
    unsigned short* dvp = a.dv + ((long)b * a.S + my_key) * a.Hkv * HD + (long)hk * HD;
#pragma unroll
    for (int d = 0; d < NDB; ++d)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int col = d * 32 + 8 * gq + 4 * hh;
        float kx[4], vx[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          kx[j] = dk[d][4 * gq + j];
          vx[j] = dv[d][4 * gq + j];
        }
        store_bf16x4(dkp + col, kx, a.scale);
        store_bf16x4(dvp + col, vx, 1.f);
      }
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
  constexpr int CPR = HD / 8;
  constexpr int LD_ITERS = DQ_KB * CPR / 256;
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * DQ_KB * ROWB];
  unsigned char* Ks = smem;                // tr image: row reads (S^T) and column reads (dQ^T)
  unsigned char* Vs = smem + DQ_KB * ROWB;  // row image

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int nqb = (a.S + DQ_QB - 1) / DQ_QB;
  const int BH = a.B * a.Hq;
  const int bh = blockIdx.x % BH;
  const int qblk = nqb - 1 - (int)(blockIdx.x / BH);  // heaviest first
  const int b = bh / a.Hq, hq = bh % a.Hq;
  const int hk = hq / (a.Hq / a.Hkv);
  const int q_row0 = qblk * DQ_QB + wave * 32;
  const int my_q = q_row0 + r;
  const int qc = min(my_q, a.S - 1);

  const unsigned short* Kp = a.k + b * a.k_sb + hk * a.k_sh;
  const unsigned short* Vp = a.v + b * a.v_sb + hk * a.v_sh;

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
  const float dlt = a.delta[rc];

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
    w_min = ds[min(q_row0, a.S - 1)];
    w_max = ds[min(q_row0 + 31, a.S - 1)];
    t0 = ds[min(qblk * DQ_QB, a.S - 1)] / DQ_KB;
  }

  uint4 kst[LD_ITERS], vst[LD_ITERS];
  auto issue = [&](int t) {
#pragma unroll
    for (int it = 0; it < LD_ITERS; ++it) {
      const int c = tid + 256 * it;
      const int row = c / CPR, ch = c % CPR;
      const int key = min(t * DQ_KB + row, a.S - 1);  // keys past S: masked
      kst[it] = gload16(Kp + (long)key * a.k_ss + ch * 8);
      vst[it] = gload16(Vp + (long)key * a.v_ss + ch * 8);
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int it = 0; it < LD_ITERS; ++it) {
      const int c = tid + 256 * it;
      const int row = c / CPR, ch = c % CPR;
      *reinterpret_cast<uint4*>(Ks + tr_off<HD>(row, ch)) = kst[it];
      *reinterpret_cast<uint4*>(Vs + row_off<HD>(row, ch)) = vst[it];
    }
  };

  if (t0 < ntiles) issue(t0);
  for (int t = t0; t < ntiles; ++t) {
    __syncthreads();  // all waves finished reading the previous tile
    commit();
    __syncthreads();
    if (t + 1 < ntiles) issue(t + 1);  // overlaps the MFMAs below
    const int kv0 = t * DQ_KB;
    if (CAUSAL && kv0 > q_row0 + 31) continue;  // tile entirely above this wave's diagonal
    if (DOC && kv0 + DQ_KB <= w_min) continue;  // tile entirely before every row's document
    const bool need_mask = (CAUSAL && kv0 + DQ_KB - 1 > q_row0) || (kv0 + DQ_KB > a.S) || (DOC && kv0 < w_max);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      // ---- S^T = K Q^T, dP^T = V dO^T   (key on regs, q on lane)
      f32x16 s, dp;
#pragma unroll
      for (int i = 0; i < 16; ++i) s[i] = dp[i] = 0.f;
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const bf16x8_t kfr = lds_read_b128(Ks, tr_off<HD>(kb * 32 + r, 2 * ks + hh));
        s = mfma32(kfr, qf[ks], s);
        const bf16x8_t vfr = lds_read_b128(Vs, row_off<HD>(kb * 32 + r, 2 * ks + hh));
        dp = mfma32(vfr, df[ks], dp);
      }
      float dsv[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float pv = fast_exp2(s[i] * a.scale_log2 + nlse2);
        if (need_mask) {
          const int key = kv0 + kb * 32 + acc_row(i, hh);
          if ((CAUSAL && key > my_q) || key >= a.S || (DOC && key < my_start)) pv = 0.f;
        }
        dsv[i] = pv * (dp[i] - dlt);
      }
      // ---- dQ^T += K^T dS^T   (sum over keys = the registers of dS^T)
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const bf16x8_t sbf = to_bf16x8(dsv + 8 * st);
#pragma unroll
        for (int d = 0; d < NDB; ++d) {
          const bf16x8_t kt = tr_frag<HD>(Ks, kb * 32 + 16 * st, d * 32, lane);
          dq[d] = mfma32(kt, sbf, dq[d]);
        }
      }
    }
  }
  // ---- dQ = scale * (dQ^T)^T: lane = q row, registers = d
  if (my_q < a.S) {
    unsigned short* Op = a.dq + ((long)b * a.S + my_q) * a.Hq * HD + (long)hq * HD;
#pragma unroll
    for (int d = 0; d < NDB; ++d)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float x[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) x[j] = dq[d][4 * g + j];
        store_bf16x4(Op + d * 32 + 8 * g + 4 * hh, x, a.scale);
      }
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
                 (float)scale, (float)(scale * 1.4426950408889634), nullptr};
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
  const long threads = (long)B * S * Hq * (D / 8);
  if (D == 128)
    hipLaunchKernelGGL(delta_kernel<128>, dim3((threads + 255) / 256), dim3(256), 0, s, bf_ptr(dout), bf_ptr(o),
                       delta.data_ptr<float>(), B, S, Hq, dout.stride(0), dout.stride(1), dout.stride(2), o.stride(0),
                       o.stride(1), o.stride(2));
  else
    hipLaunchKernelGGL(delta_kernel<64>, dim3((threads + 255) / 256), dim3(256), 0, s, bf_ptr(dout), bf_ptr(o),
                       delta.data_ptr<float>(), B, S, Hq, dout.stride(0), dout.stride(1), dout.stride(2), o.stride(0),
                       o.stride(1), o.stride(2));
  BwdArgs a = make_args(dout, q, k, v, lse, delta, dq, dk, dv, scale);
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

// timing-only entry for tools/attn_ablate.py (causal, no documents): abl 0 = both kernels,
// 1 = dK/dV kernel only, 2 = dQ kernel only, 3 / 4 = dK/dV schedule variants 1 / 2.  ``delta`` is taken as given.
void fa_bwd_ablate(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                   const at::Tensor& delta, const at::Tensor& lse, at::Tensor& dq, at::Tensor& dk, at::Tensor& dv,
                   int64_t abl) {
  const int D = q.size(3);
  LLMCTL_CHECK(D == 64 || D == 128, "fa_bwd_ablate: head_dim 64 or 128");
  LLMCTL_CHECK(dq.scalar_type() == at::kBFloat16 && dq.sizes() == q.sizes() && dk.sizes() == k.sizes() &&
                   dv.sizes() == k.sizes() && delta.numel() == lse.numel(),
               "fa_bwd_ablate: bf16 dq/dk/dv, fp32 delta");
  const c10::DeviceGuard g(q.device());
  BwdArgs a = make_args(dout, q, k, v, lse, delta, dq, dk, dv, 1.0 / std::sqrt((double)D));
  if (abl == 3 || abl == 4) {
    LLMCTL_CHECK(D == 128, "fa_bwd_ablate: schedule variants at head_dim 128");
    const int nkb = (a.S + KV_KB - 1) / KV_KB;
    const dim3 grid((unsigned)(a.B * a.Hkv * nkb));
    if (abl == 3) hipLaunchKernelGGL((fa_bwd_dkv_kernel<128, true, false, 1>), grid, dim3(256), 0, stream(), a);
    else hipLaunchKernelGGL((fa_bwd_dkv_kernel<128, true, false, 2>), grid, dim3(256), 0, stream(), a);
    return;
  }
  dispatch_bwd(a, D, true, false, stream(), abl != 1, abl != 2);
}

TORCH_LIBRARY_IMPL(llmctl, CUDA, m) {
  m.impl("flash_attn_bwd", &flash_attn_bwd);
  m.impl("fa_bwd_ablate", &fa_bwd_ablate);
}

}  // namespace llmctl
