// Flash-attention backward (causal / full, GQA) for gfx950 — MFMA 32x32x16 bf16.
//
// Algorithm (CDNA guide App. B "Attention backward"): recompute P from Q, K and the
// forward's LSE; five MFMA products per tile:
//     S = Q K^T,  dP = dO V^T,  dV^T += dO^T P,  dK^T += Q^T dS,  dQ += dS K
// Structure:
//   * workgroup = 4 waves = 128 keys of one (batch, kv-head); wave w owns keys
//     [32w, 32w+32) and keeps dK^T / dV^T for them in registers across ALL query tiles and
//     ALL q-heads of its GQA group (no cross-workgroup sum for dK/dV);
//   * keys on the MFMA lane: S and dP accumulators are directly the B operands of the dV^T
//     and dK^T products (accumulator-as-operand, no LDS round trip);
//   * one LDS image per tile for K, V, Q, dO (XOR-swizzled "tr image": conflict-free for
//     both ds_read_b128 row reads and ds_read_b64_tr_b16 transposed reads, guide T10);
//   * only dS crosses LDS (as dS^T, 64-B rows), for dQ = dS K, which is split over the 4
//     waves by d-block and accumulated with fp32 atomics (two 128-B row segments per
//     wave-instruction = the full atomic rate, guide "Global float atomics");
//   * LSE / delta are folded in as per-row constants; exp2 domain throughout.
// A pre-kernel computes delta = rowsum(dO*O) and a post-kernel converts dQ (fp32) to bf16.
#include "attn_common.h"

namespace llmctl {
using namespace attn;
namespace {

constexpr int KBLK = 128;  // keys per workgroup
constexpr int QT = 32;     // query rows per iteration

struct BwdArgs {
  const unsigned short *q, *k, *v, *o, *dout;
  const float* lse;    // [B,Hq,S] natural log
  const float* delta;  // [B,Hq,S]
  float* dq_acc;       // [B,S,Hq,HD] fp32 (contiguous)
  unsigned short *dk, *dv;  // [B,S,Hkv,HD] contiguous
  int B, S, Hq, Hkv;
  long q_sb, q_ss, q_sh, k_sb, k_ss, k_sh, v_sb, v_ss, v_sh, o_sb, o_ss, o_sh, do_sb, do_ss, do_sh;
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

__global__ __launch_bounds__(256) void f32_to_bf16_kernel(const float* __restrict__ x, unsigned short* __restrict__ y,
                                                           long n8) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n8) return;
  float v[8];
  *reinterpret_cast<float4*>(v) = reinterpret_cast<const float4*>(x + i * 8)[0];
  *reinterpret_cast<float4*>(v + 4) = reinterpret_cast<const float4*>(x + i * 8)[1];
  store8(y + i * 8, v);
}

// ABL: timing ablations for tools/attn_bench.py (results wrong): 1 no dQ atomics,
// 2 no dQ product (and no dS^T exchange), 4 no Q/dO prefetch (tile 0 reused)
template <int HD, bool CAUSAL, int ABL = 0, bool DOC = false>
__global__ __launch_bounds__(256, 1) void fa_bwd_kernel(BwdArgs a) {
  constexpr int NKS = HD / 16;
  constexpr int NDB = HD / 32;
  constexpr int ROWB = HD * 2;
  constexpr int CPR = HD / 8;
  constexpr int KV_ITERS = KBLK * CPR / 256;  // 8 for HD=128
  constexpr int Q_ITERS = QT * CPR / 256;     // 2 for HD=128
  constexpr int DST_ROWB = QT * 2;            // dS^T rows: 32 q * 2 B = 64 B
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * KBLK * ROWB + 4 * QT * ROWB + KBLK * DST_ROWB +
                                                             6 * QT * 4];
  unsigned char* Ks = smem;
  unsigned char* Vs = Ks + KBLK * ROWB;
  unsigned char* Qbuf = Vs + KBLK * ROWB;       // [2][QT][HD] double-buffered Q tiles
  unsigned char* Dbuf = Qbuf + 2 * QT * ROWB;   // [2][QT][HD] double-buffered dO tiles
  unsigned char* St = Dbuf + 2 * QT * ROWB;     // dS^T [key][q]
  float* lse_buf = reinterpret_cast<float*>(St + KBLK * DST_ROWB);  // [2][QT]
  float* del_buf = lse_buf + 2 * QT;                                 // [2][QT]
  int* doc_buf = reinterpret_cast<int*>(del_buf + 2 * QT);           // [2][QT] (packed documents)

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int BH = a.B * a.Hkv;
  const int bh = blockIdx.x % BH;
  const int kblk = blockIdx.x / BH;  // small kblk = most query tiles under causal: dispatched first
  const int b = bh / a.Hkv, hk = bh % a.Hkv;
  const int group = a.Hq / a.Hkv;
  const int k0 = kblk * KBLK;
  const int wkey0 = k0 + wave * 32;  // this wave's first key
  const int my_key = wkey0 + r;

  const unsigned short* Kp = a.k + b * a.k_sb + hk * a.k_sh;
  const unsigned short* Vp = a.v + b * a.v_sb + hk * a.v_sh;

  // ---- stage this block's K and V (tr images) once
#pragma unroll
  for (int it = 0; it < KV_ITERS; ++it) {
    const int c = tid + 256 * it;
    const int row = c / CPR, ch = c % CPR;
    const int key = k0 + row;
    uint4 kk = make_uint4(0, 0, 0, 0), vv = make_uint4(0, 0, 0, 0);
    if (key < a.S) {
      kk = gload16(Kp + (long)key * a.k_ss + ch * 8);
      vv = gload16(Vp + (long)key * a.v_ss + ch * 8);
    }
    *reinterpret_cast<uint4*>(Ks + tr_off<HD>(row, ch)) = kk;
    *reinterpret_cast<uint4*>(Vs + tr_off<HD>(row, ch)) = vv;
  }

  f32x16 dk[NDB], dv[NDB];
#pragma unroll
  for (int d = 0; d < NDB; ++d)
#pragma unroll
    for (int i = 0; i < 16; ++i) dk[d][i] = dv[d][i] = 0.f;

  // flattened (q-head of the GQA group, query tile) sequence; the next tile's Q / dO / lse /
  // delta are prefetched into registers while the current one is computed (register staging,
  // guide T14) and written to the other LDS buffer after it
  const int q_start = CAUSAL ? (k0 / QT) * QT : 0;
  int q_end = a.S;
  if constexpr (DOC) {
    // queries whose document starts after this block's last key see none of its keys:
    // q_end = first position with doc_start > k0 + KBLK - 1 (doc_start is non-decreasing)
    const int* ds = a.doc + (long)b * a.S;
    int lo = min(k0 + KBLK, a.S), hi = a.S;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (ds[mid] > k0 + KBLK - 1) hi = mid;
      else lo = mid + 1;
    }
    q_end = lo;
  }
  const int nq = q_end > q_start ? (q_end - q_start + QT - 1) / QT : 0;
  const int ntiles = group * nq;
  uint4 pq[Q_ITERS], pd[Q_ITERS];
  float pl = 0.f, pdl = 0.f;
  int pds = 0;
  // unconditional loads (rows past S clamped to S-1: their P is masked to 0, so they add
  // nothing): no zero-init + branch, which made hipcc drain vmcnt at every fetch
  auto fetch = [&](int t) {
    const int g = t / nq;
    const int q0 = q_start + (t - g * nq) * QT;
    const int hq = hk * group + g;
    const unsigned short* Qp = a.q + b * a.q_sb + hq * a.q_sh;
    const unsigned short* Dp = a.dout + b * a.do_sb + hq * a.do_sh;
#pragma unroll
    for (int it = 0; it < Q_ITERS; ++it) {
      const int c = tid + 256 * it;
      const int row = c / CPR, ch = c % CPR;
      const int qq = min(q0 + row, a.S - 1);
      pq[it] = gload16(Qp + (long)qq * a.q_ss + ch * 8);
      pd[it] = gload16(Dp + (long)qq * a.do_ss + ch * 8);
    }
    if (tid < QT) {
      const int qq = min(q0 + tid, a.S - 1);
      const long base = ((long)b * a.Hq + hq) * a.S;
      pl = a.lse[base + qq];  // scaled to log2 at commit (no use of the load here)
      pdl = a.delta[base + qq];
      if constexpr (DOC) pds = a.doc[(long)b * a.S + qq];
    }
  };
  auto commit = [&](int buf) {
    unsigned char* Qs = Qbuf + buf * QT * ROWB;
    unsigned char* Ds = Dbuf + buf * QT * ROWB;
#pragma unroll
    for (int it = 0; it < Q_ITERS; ++it) {
      const int c = tid + 256 * it;
      const int row = c / CPR, ch = c % CPR;
      *reinterpret_cast<uint4*>(Qs + tr_off<HD>(row, ch)) = pq[it];
      *reinterpret_cast<uint4*>(Ds + tr_off<HD>(row, ch)) = pd[it];
    }
    if (tid < QT) {
      lse_buf[buf * QT + tid] = pl * 1.4426950408889634f;
      del_buf[buf * QT + tid] = pdl;
      if constexpr (DOC) doc_buf[buf * QT + tid] = pds;
    }
  };
  if (ntiles > 0) {
    fetch(0);
    commit(0);
  }
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    const int g = t / nq;
    const int q0 = q_start + (t - g * nq) * QT;
    const int hq = hk * group + g;
    float* dq_p = a.dq_acc + (long)b * a.S * a.Hq * HD + (long)hq * HD;
    const unsigned char* Qs = Qbuf + buf * QT * ROWB;
    const unsigned char* Ds = Dbuf + buf * QT * ROWB;
    const float* lse_s = lse_buf + buf * QT;
    const float* del_s = del_buf + buf * QT;
    const int* doc_s = doc_buf + buf * QT;
    // packed documents: the tile's smallest / largest document start (non-decreasing)
    const int dmin = DOC ? doc_s[0] : 0, dmax = DOC ? doc_s[QT - 1] : 0;
    if (!(ABL & 4) && t + 1 < ntiles) fetch(t + 1);  // in flight during this tile's MFMAs

    const bool active = !(CAUSAL && wkey0 > q0 + QT - 1) && wkey0 < a.S && !(DOC && wkey0 + 31 < dmin);
    float pbuf[16], dsbuf[16];
    if (active) {
      // ---- S = Q K^T and dP = dO V^T   (q on regs, key on lane)
      f32x16 s, dp;
#pragma unroll
      for (int i = 0; i < 16; ++i) s[i] = dp[i] = 0.f;
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const bf16x8_t qa = lds_read_b128(Qs, tr_off<HD>(r, 2 * ks + hh));
        const bf16x8_t kb = lds_read_b128(Ks, tr_off<HD>(wave * 32 + r, 2 * ks + hh));
        s = mfma32(qa, kb, s);
        const bf16x8_t da = lds_read_b128(Ds, tr_off<HD>(r, 2 * ks + hh));
        const bf16x8_t vb = lds_read_b128(Vs, tr_off<HD>(wave * 32 + r, 2 * ks + hh));
        dp = mfma32(da, vb, dp);
      }
      const bool need_mask = (CAUSAL && wkey0 + 31 > q0) || (q0 + QT > a.S) || (wkey0 + 32 > a.S) ||
                             (DOC && wkey0 < dmax);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int qi = acc_row(i, hh);
        float p = fast_exp2(s[i] * a.scale_log2 - lse_s[qi]);
        if (need_mask) {
          const int qq = q0 + qi;
          if ((CAUSAL && my_key > qq) || qq >= a.S || my_key >= a.S || (DOC && my_key < doc_s[qi])) p = 0.f;
        }
        pbuf[i] = p;
        dsbuf[i] = p * (dp[i] - del_s[qi]) * a.scale;
      }
      // ---- dV^T += dO^T P ; dK^T += Q^T dS
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const bf16x8_t pb = to_bf16x8(pbuf + 8 * st);
        const bf16x8_t sb = to_bf16x8(dsbuf + 8 * st);
#pragma unroll
        for (int d = 0; d < NDB; ++d) {
          const bf16x8_t da = tr_frag<HD>(Ds, 16 * st, d * 32, lane);
          dv[d] = mfma32(da, pb, dv[d]);
          const bf16x8_t qa = tr_frag<HD>(Qs, 16 * st, d * 32, lane);
          dk[d] = mfma32(qa, sb, dk[d]);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) dsbuf[i] = 0.f;
    }
    // ---- dS^T -> LDS [key][q] (64-B rows): lane = key, 4 groups of 4 contiguous q
    {
      unsigned char* rowp = St + (wave * 32 + r) * DST_ROWB;
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int qc = 8 * gq + 4 * hh;
        unsigned short w4[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) w4[j] = f2bf(dsbuf[4 * gq + j]);
        *reinterpret_cast<uint2*>(rowp + qc * 2) =
            make_uint2((unsigned)w4[0] | ((unsigned)w4[1] << 16), (unsigned)w4[2] | ((unsigned)w4[3] << 16));
      }
    }
    lds_sync();
    // ---- dQ[q][d] += dS K over this block's 128 keys; waves split the d-blocks
    {
      constexpr int WPD = 4 / NDB;  // waves per d-block (1 for HD=128, 2 for HD=64)
      const int d = wave / WPD;
      const int kpart = wave % WPD;
      constexpr int KSTEPS = KBLK / 16 / WPD;
      // skip if every key of this block is above this q tile's diagonal (all dS zero)
      if (!(ABL & 2) && !(CAUSAL && k0 > q0 + QT - 1) && !(DOC && k0 + KBLK - 1 < dmin)) {
        f32x16 acc;
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
        for (int ks = 0; ks < KSTEPS; ++ks) {
          const int key0 = (kpart * KSTEPS + ks) * 16;
          // A = dS[q][key]: from dS^T image X[key][q] (64-B rows, plain layout)
          const int i16 = lane & 15, qq4 = i16 >> 2, p = i16 & 3;
          const int col = 16 * ((lane >> 4) & 1) + 4 * p;  // q column
          const int r1 = key0 + 8 * hh + qq4;
          s4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(St + r1 * DST_ROWB + col * 2));
          s4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(St + (r1 + 4) * DST_ROWB + col * 2));
          s8_t av = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          const bf16x8_t af = __builtin_bit_cast(bf16x8_t, av);
          // B = K[key][d] with d on the lane
          const bf16x8_t bf = tr_frag_nat<HD>(Ks, key0, d * 32, lane);
          acc = mfma32(af, bf, acc);
        }
        // the next tile's Q / dO go to the other buffer BEFORE the atomics are issued, so
        // the wait for the prefetch loads is not a wait for the (younger) atomics; that
        // buffer was last read during tile t-1, before this tile's first barrier
        if (!(ABL & 4) && t + 1 < ntiles) commit(buf ^ 1);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int qq = q0 + acc_row(i, hh);
          if constexpr (ABL & 1) {
            asm volatile("" ::"v"(acc[i]));
          } else {
            // unconditional (rows past S add 0 to row S-1): a branch per atomic makes
            // hipcc's vmcnt accounting assume they may not exist and drain them early
            atomicAdd(dq_p + (long)min(qq, a.S - 1) * a.Hq * HD + d * 32 + r, qq < a.S ? acc[i] : 0.f);
          }
        }
      } else if (!(ABL & 4) && t + 1 < ntiles) {
        commit(buf ^ 1);
      }
    }
    lds_sync();  // LDS-only: the dQ atomics and the next tile's loads stay in flight
  }
  // ---- write dK, dV (bf16) for this wave's keys: lane = key, regs = d
  if (my_key < a.S) {
    unsigned short* dkp = a.dk + ((long)b * a.S + my_key) * a.Hkv * HD + (long)hk * HD;
    unsigned short* dvp = a.dv + ((long)b * a.S + my_key) * a.Hkv * HD + (long)hk * HD;
#pragma unroll
    for (int d = 0; d < NDB; ++d)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int col = d * 32 + 8 * gq + 4 * hh;
        unsigned short k4[4], v4[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          k4[j] = f2bf(dk[d][4 * gq + j]);
          v4[j] = f2bf(dv[d][4 * gq + j]);
        }
        *reinterpret_cast<uint2*>(dkp + col) =
            make_uint2((unsigned)k4[0] | ((unsigned)k4[1] << 16), (unsigned)k4[2] | ((unsigned)k4[3] << 16));
        *reinterpret_cast<uint2*>(dvp + col) =
            make_uint2((unsigned)v4[0] | ((unsigned)v4[1] << 16), (unsigned)v4[2] | ((unsigned)v4[3] << 16));
      }
  }
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
  LLMCTL_CHECK(dout.sizes() == q.sizes() && o.sizes() == q.sizes() && k.sizes() == v.sizes(), "shape mismatch");
  LLMCTL_CHECK(lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.numel() == (long)B * Hq * S,
               "lse must be contiguous fp32 [B,Hq,S]");
  for (const at::Tensor* t : {&dout, &q, &k, &v, &o})
    LLMCTL_CHECK(t->scalar_type() == at::kBFloat16 && t->stride(3) == 1 && t->stride(0) % 8 == 0 &&
                     t->stride(1) % 8 == 0 && t->stride(2) % 8 == 0 &&
                     (reinterpret_cast<uintptr_t>(t->data_ptr()) & 15) == 0,
                 "flash_attn_bwd: bf16, d-contiguous, 16-B aligned rows");
  const c10::DeviceGuard g(q.device());
  auto dq_acc = at::zeros({B, S, Hq, D}, q.options().dtype(at::kFloat));
  auto delta = at::empty({B, Hq, S}, q.options().dtype(at::kFloat));
  auto dk = at::empty({B, S, Hkv, D}, q.options());
  auto dv = at::empty({B, S, Hkv, D}, q.options());
  auto dq = at::empty({B, S, Hq, D}, q.options());
  if ((long)B * S * Hq == 0) return {dq, dk, dv};
  auto s = stream();
  const long R = (long)B * S * Hq;
  const long threads = R * (D / 8);
  if (D == 128)
    hipLaunchKernelGGL(delta_kernel<128>, dim3((threads + 255) / 256), dim3(256), 0, s, bf_ptr(dout), bf_ptr(o),
                       delta.data_ptr<float>(), B, S, Hq, dout.stride(0), dout.stride(1), dout.stride(2), o.stride(0),
                       o.stride(1), o.stride(2));
  else
    hipLaunchKernelGGL(delta_kernel<64>, dim3((threads + 255) / 256), dim3(256), 0, s, bf_ptr(dout), bf_ptr(o),
                       delta.data_ptr<float>(), B, S, Hq, dout.stride(0), dout.stride(1), dout.stride(2), o.stride(0),
                       o.stride(1), o.stride(2));
  BwdArgs a{bf_ptr(q), bf_ptr(k), bf_ptr(v), bf_ptr(o), bf_ptr(dout), lse.data_ptr<float>(), delta.data_ptr<float>(),
            dq_acc.data_ptr<float>(), bf_mut(dk), bf_mut(dv), B, S, Hq, Hkv,
            q.stride(0), q.stride(1), q.stride(2), k.stride(0), k.stride(1), k.stride(2),
            v.stride(0), v.stride(1), v.stride(2), o.stride(0), o.stride(1), o.stride(2),
            dout.stride(0), dout.stride(1), dout.stride(2), (float)scale, (float)(scale * 1.4426950408889634),
            nullptr};
  const int nkb = (S + KBLK - 1) / KBLK;
  dim3 grid((unsigned)(B * Hkv * nkb)), block(256);
  if (doc_start.has_value() && doc_start->defined()) {
    const at::Tensor& ds = *doc_start;
    LLMCTL_CHECK(causal && ds.is_cuda() && ds.scalar_type() == at::kInt && ds.is_contiguous() && ds.dim() == 2 &&
                     ds.size(0) == B && ds.size(1) == S,
                 "flash_attn_bwd: doc_start must be contiguous int32 [B,S] (causal)");
    a.doc = ds.data_ptr<int>();
    if (D == 128) hipLaunchKernelGGL((fa_bwd_kernel<128, true, 0, true>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((fa_bwd_kernel<64, true, 0, true>), grid, block, 0, s, a);
  } else if (D == 128) {
    if (causal) hipLaunchKernelGGL((fa_bwd_kernel<128, true>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((fa_bwd_kernel<128, false>), grid, block, 0, s, a);
  } else {
    if (causal) hipLaunchKernelGGL((fa_bwd_kernel<64, true>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((fa_bwd_kernel<64, false>), grid, block, 0, s, a);
  }
  const long n8 = dq.numel() / 8;
  hipLaunchKernelGGL(f32_to_bf16_kernel, dim3((n8 + 255) / 256), dim3(256), 0, s, dq_acc.data_ptr<float>(),
                     bf_mut(dq), n8);
  return {dq, dk, dv};
}

// timing-only ablation entry (HD=128, causal): same launch as flash_attn_bwd's main kernel
void fa_bwd_ablate(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                   const at::Tensor& o, const at::Tensor& lse, at::Tensor& dq_acc, at::Tensor& dk, at::Tensor& dv,
                   int64_t abl) {
  const int B = q.size(0), S = q.size(1), Hq = q.size(2), D = q.size(3), Hkv = k.size(2);
  LLMCTL_CHECK(D == 128, "fa_bwd_ablate: D=128 only");
  const c10::DeviceGuard g(q.device());
  BwdArgs a{bf_ptr(q), bf_ptr(k), bf_ptr(v), bf_ptr(o), bf_ptr(dout), lse.data_ptr<float>(), lse.data_ptr<float>(),
            dq_acc.data_ptr<float>(), bf_mut(dk), bf_mut(dv), B, S, Hq, Hkv,
            q.stride(0), q.stride(1), q.stride(2), k.stride(0), k.stride(1), k.stride(2),
            v.stride(0), v.stride(1), v.stride(2), o.stride(0), o.stride(1), o.stride(2),
            dout.stride(0), dout.stride(1), dout.stride(2), 0.088f, 0.127f, nullptr};
  dim3 grid((unsigned)(B * Hkv * ((S + KBLK - 1) / KBLK))), block(256);
  auto s = stream();
  switch (abl) {
    case 0: hipLaunchKernelGGL((fa_bwd_kernel<128, true, 0>), grid, block, 0, s, a); break;
    case 1: hipLaunchKernelGGL((fa_bwd_kernel<128, true, 1>), grid, block, 0, s, a); break;
    case 2: hipLaunchKernelGGL((fa_bwd_kernel<128, true, 2>), grid, block, 0, s, a); break;
    case 4: hipLaunchKernelGGL((fa_bwd_kernel<128, true, 4>), grid, block, 0, s, a); break;
    default: hipLaunchKernelGGL((fa_bwd_kernel<128, true, 6>), grid, block, 0, s, a); break;
  }
}

TORCH_LIBRARY_IMPL(llmctl, CUDA, m) {
  m.impl("flash_attn_bwd", &flash_attn_bwd);
  m.impl("fa_bwd_ablate", &fa_bwd_ablate);
}

}  // namespace llmctl
