// bf16 MFMA GEMM, 256x256 tile, 64-deep K-tiles, half-tile LDS-DMA pipeline (gfx950).
//
//   C[M,N] (+)= sum_k A(m,k) * B(n,k)        fp32 accumulate, bf16 in/out
//
// Operand storage per template flag, as in gemm_bf16.hip: "K-contiguous" (A [M][K], B [N][K])
// or "K-major" (A [K][M], B [K][N]); the three products of a linear layer map to
//   forward  y  = x  W^T :  A = x [T][in], B = W [out][in]                  (AT=0, BT=0)
//   dgrad    dx = dy W   :  A = dy [T][out], B(n=in,k=out) = W [out][in]     (AT=0, BT=1)
//   wgrad    dW = dy^T x :  A(m=out,k=t) = dy [t][out], B(n=in,k=t) = x [t][in] (AT=1, BT=1)
//
// Why a second kernel family: gemm_bf16.hip stages 32-deep K-tiles, so a K-contiguous operand
// row contributes 64 B per tile — every 128-B line is fetched in two halves by two tiles, and
// that layout ran at 1.17-1.21 PF where the K-major (full 512-B rows) layouts reached 1.23-1.36
// (profiles/gemm_bench_r1.json).  Here a K-tile is 64 deep: a K-contiguous row is one full
// 128-B line per tile, a K-major image row is 256 B.
//
// Structure (CDNA guide §5 "256² 8-phase template", re-derived for this tile):
//   * 8 waves = 2 (M) x 4 (N); wave (wr, wc) owns the 128x64 output block at rows wr*128,
//     cols wc*64 = 8x4 tiles of mfma_f32_16x16x32_bf16 (128 accumulator registers), computed
//     transposed (B fragment as the MFMA row operand) so a lane holds 4 consecutive columns.
//   * A K-tile is staged as four 16-KB half-tiles, each filled by 2 LDS-DMA instructions per
//     thread (buffer_load_dwordx4 ... lds, lane-linear image, swizzle applied to the SOURCE):
//        A_lo = rows {0..63, 128..191}   (m-tiles 0-3 of both wave rows)
//        A_hi = rows {64..127, 192..255} (m-tiles 4-7)
//        B_h0 = cols 0..127 (waves wc 0,1), B_h1 = cols 128..255 (waves wc 2,3)
//     Two K-tile buffers (128 KB of LDS).
//   * 4 phases per K-tile, 16 MFMAs each (one 64x32 quadrant x K=64):
//        j=0  read A_lo frags (m 0-3) + B frags n 0-1 -> quadrant (m 0-3, n 0-1)
//        j=1  read B frags n 2-3                      -> (m 0-3, n 2-3)
//        j=2  read A_hi frags (m 4-7)                 -> (m 4-7, n 2-3)
//        j=3  (no reads)                              -> (m 4-7, n 0-1)
//     Each phase issues ONE half-tile of the stream (2 DMA instructions) right after its first
//     barrier:  j=0: B_h1(t+1)  j=1: A_hi(t+1)  j=2: A_lo(t+2)  j=3: B_h0(t+2).
//     Every slot is restaged >= 2 phases after its last read (WAR); the counted waits
//        j=1: vmcnt(6)  (retires A_hi(t), read at j=2)
//        j=3: vmcnt(4)  (retires A_lo/B_h0/B_h1 of t+1, read at j=0 of t+1)
//     sit before the first barrier of the phase BEFORE the read (RAW across waves), so at
//     least 2-3 half-tiles stay in flight across every barrier; raw s_barrier only.
//   * Two wave groups (wr = 0 / 1, one wave of each per SIMD) run one barrier apart: one
//     group's LDS fragment reads overlap the other group's MFMAs (ping-pong).
//   * Stream items past the last K-tile re-load the last K-tile (clamped source) into slots
//     nobody reads again, so the wait counts never change in the tail.
//   * XCD-aware bijective block remap + grouped tile order (GROUP tile-rows).
//   * Tail split ("split-K on the last round"): with one 512-thread workgroup per CU, a grid of
//     T tiles runs ceil(T / CUs) rounds and the last one is partly idle (GPT-7B wgrad of the
//     up-projection: 1376 tiles = 5.375 rounds, 10 % of its time).  The tiles of the partial
//     round are cut into S K-ranges; those items write fp32 partials to a workspace and a
//     reduction kernel applies the epilogue, so the last round costs ~1/S of a tile.
#include "attn_common.h"

namespace llmctl {
using namespace attn;
namespace {

using f32x4_t = __attribute__((ext_vector_type(4))) float;
using s2_t = __attribute__((ext_vector_type(2))) unsigned int;
using i32x4_t = __attribute__((ext_vector_type(4))) int;

constexpr int TM = 256, TN = 256, TK = 64;
constexpr int HALF = 16384;       // bytes per half-tile image
constexpr int BUF = 4 * HALF;     // one K-tile: A_lo, A_hi, B_h0, B_h1
constexpr int NTHR = 512;
enum : int { A_LO = 0, A_HI = 1, B_H0 = 2, B_H1 = 3 };

// epilogues
// EPI_SWIGLU_BWD (down-projection data gradient): C = dAct is not stored; with gate / up read from
// aux = gu [M, 2N] (ld = ldc), the epilogue writes dgate to C[:, n] and dup to C[:, N + n] (C = dgu),
// i.e. the SwiGLU backward rides on the GEMM's store pass (no dAct round trip through HBM)
// EPI_SWIGLU_FWD (gate/up projection, forward layout, serving prefill): output tile tn covers gate
// rows [128 tn, 128 tn + 128) of B = W_up [2F, K] in its left half and the matching up rows
// F + [128 tn, ...) in its right half (the second B half-tile reads through its own buffer
// resource); the up accumulators cross to the gate waves through LDS and only act = silu(g) * u
// [M, F] is stored (C, ldc = F) — no gu tensor, no separate SwiGLU pass
// EPI_STORE_F32 / EPI_ACC_F32 (fp32 main gradients, wgrad layout): C is fp32 (args.c reinterpreted
// as float*, ldc in floats): the weight gradient is written / accumulated in fp32, never rounded
// to bf16 between micro-steps
// Fused training-forward epilogues (one-shot kernel; B fragment slots remapped so each wave owns
// both columns of every pair it combines — no cross-wave exchange):
// EPI_ROPE_QKV: QKV projection (D = 128: a 256-column tile = 2 heads).  Wave wc owns head
//   (wc >> 1)'s dims (wc & 1) * 32 + [0, 32) and the same + 64, i.e. both halves of its rotation
//   pairs; the epilogue rounds to bf16, applies RoPE to q / k heads (cos / sin tables [P][64],
//   position = pos[t] or t % seq) and stores q [T, nq, D], k / v [T, nkv, D] separately — the
//   rope_qkv_fwd pass and its re-read of qkv disappear.
// EPI_UP_SWIGLU: gate/up projection with the gate rows 128 tn.. (B_h0) and the matching up rows
//   F + 128 tn.. (B_h1, as EPI_SWIGLU_FWD) in one tile; wave wc owns gate cols wc * 32 + [0, 32)
//   and the same up cols; stores gu [T, 2F] (kept for the backward) AND act = silu(g) * u [T, F]
//   — the swiglu_fwd pass and its re-read of gu disappear.
enum : int {
  EPI_STORE = 0, EPI_ACC = 1, EPI_SWIGLU_BWD = 2, EPI_SWIGLU_FWD = 3, EPI_STORE_F32 = 4, EPI_ACC_F32 = 5,
  EPI_ROPE_QKV = 6, EPI_UP_SWIGLU = 7
};
constexpr bool epi_f32(int e) { return e == EPI_STORE_F32 || e == EPI_ACC_F32; }
template <int V>
using K_ = std::integral_constant<int, V>;

struct G64Args {
  const unsigned short* a;
  const unsigned short* b;
  unsigned short* c;
  long lda, ldb, ldc;
  int M, N, K;
  int tiles_m, tiles_n;
  int n_main;   // tiles computed whole (blocks [0, n_main)); the rest are split
  int splits;   // K-ranges per split tile (1: no split items)
  int kt_part;  // K-tiles per split item (even)
  float* ws;    // [n_tail][splits][256][256] fp32 partials
  const unsigned short* aux;  // EPI_SWIGLU_BWD: gu [M, 2N], leading dimension ldc
  // fused forward epilogues
  unsigned short* out2 = nullptr;  // EPI_ROPE_QKV: k; EPI_UP_SWIGLU: act [M, N]
  unsigned short* out3 = nullptr;  // EPI_ROPE_QKV: v
  const float* cosT = nullptr;     // EPI_ROPE_QKV: [P][64] tables
  const float* sinT = nullptr;
  const int* pos = nullptr;        // EPI_ROPE_QKV: int32 position per token (nullptr: t % seq)
  int nq = 0, nkv = 0, seq = 1;
  // RS (row-scaled forward, serving prefill with the RMSNorm folded in): C[m, :] *= rs[m] before the
  // bf16 rounding -- rs = the rows' RMSNorm rstd, the norm weight folded into B's K columns
  const float* rs = nullptr;
  // side job (SIDE > 0, wgrad of the down projection): dgu = swiglu_bwd(dact, gu), dact [T, F],
  // gu / dgu [T, 2F], E = T * F elements spread over the K-tiles of the whole grid
  const unsigned short* s_dact = nullptr;
  const unsigned short* s_gu = nullptr;
  unsigned short* s_dgu = nullptr;
  unsigned s_E = 0;
  int s_F = 0;
  // bottleneck probes (one-shot 4-wave kernel only; results are garbage): 1 = operand loads out of
  // range (no memory traffic), 2 = no workgroup barriers, 4 = no epilogue, 8 = every tile loads
  // tile (0, 0)'s operands (L2-resident), 16 = every K-tile loads K-tile 0
  int probe = 0;
  unsigned long stamp_ptr = 0;  // STAMP diagnostic build: device buffer (knob gemm_stamp_ptr)
};

// SwiGLU backward of one element: d = dL/dact, act = silu(g) * u
__device__ __forceinline__ void swiglu_bwd1(float d, float g, float u, float& dg, float& du) {
  const float sg = 1.f / (1.f + __expf(-g));
  dg = d * u * (sg * (1.f + g * (1.f - sg)));
  du = d * (g * sg);
}

// the same with a hardware reciprocal (1 ulp) instead of an IEEE division: the side job's VALU
// runs beside MFMAs, where a 10-instruction division per element would show
__device__ __forceinline__ void swiglu_bwd1_fast(float d, float g, float u, float& dg, float& du) {
  const float sg = __builtin_amdgcn_rcpf(1.f + __expf(-g));
  dg = d * u * (sg * (1.f + g * (1.f - sg)));
  du = d * (g * sg);
}

__device__ __forceinline__ f32x4_t mfma16(bf16x8_t a, bf16x8_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ i32x4_t make_rsrc(const void* base) {
  const unsigned long a = (unsigned long)base;
  i32x4_t r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(a & 0xffffffffu));
  r[1] = __builtin_amdgcn_readfirstlane((int)((a >> 32) & 0xffff));
  r[2] = -1;          // num_records: no clamping (offsets validated on the host)
  r[3] = 0x00020000;  // raw buffer, 32-bit data format
  return r;
}
// range-checked raw buffer: loads at byte offsets >= bytes return 0, stores there are dropped
__device__ __forceinline__ i32x4_t make_rsrc_n(const void* base, unsigned bytes) {
  i32x4_t r = make_rsrc(base);
  r[2] = (int)bytes;
  return r;
}
// one LDS-DMA piece: 64 lanes x 16 B -> LDS [lds_byte, +1024), lane-linear
__device__ __forceinline__ void bdma16(i32x4_t rsrc, unsigned voff, unsigned soff, unsigned lds_byte) {
  asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(voff), "s"(rsrc),
               "s"(soff), "s"(lds_byte)
               : "memory");
}

__device__ __forceinline__ void bar() { __builtin_amdgcn_s_barrier(); }
template <int N>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 40) asm volatile("s_waitcnt vmcnt(40)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// ---- half-tile images -----------------------------------------------------------------------
// row image (K-contiguous operand): [128 image rows][64 k], 128-B rows, 16-B chunk c stored at
//   c ^ ((row >> 1) & 7): each ds_read_b128 lane group (16 lanes: rows r..r+15 at two chunks)
//   lands on 16 distinct 16-B bank slots.
// tr image (K-major operand): [64 k][128 image cols], 256-B rows, 32-B segment s stored at
//   s ^ h(k), h(k) = (k & 3) | ((k >> 3) & 1) << 2: the 8 k-rows of a 32-lane
//   ds_read_b64_tr_b16 half hit 8 distinct segments (conflict-free).
__device__ __forceinline__ int swr(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ int swt(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }

// image row/col -> tile row/col of each half-tile kind (both image kinds have 128 positions)
template <int KIND>
__device__ __forceinline__ int tile_pos(int ip) {
  if constexpr (KIND == A_LO) return (ip >> 6) * 128 + (ip & 63);
  else if constexpr (KIND == A_HI) return (ip >> 6) * 128 + 64 + (ip & 63);
  else if constexpr (KIND == B_H0) return ip;
  else return 128 + ip;
}

// per-thread byte offset (relative to the operand's tile origin at k = 0) of DMA piece i
template <bool T, int KIND, int NT = NTHR>
__device__ __forceinline__ unsigned stage_voff(int i, int tid, long ld) {
  const int c = i * NT + tid;  // 16-B chunk index in the half-tile image
  if constexpr (!T) {
    const int ir = c >> 3, pc = c & 7;
    const int row = tile_pos<KIND>(ir);
    return (unsigned)(((long)row * ld + ((pc ^ swr(ir)) << 3)) * 2);
  } else {
    const int k = c >> 4, pc = c & 15;
    const int seg = (pc >> 1) ^ swt(k);
    const int col = tile_pos<KIND>(seg * 16 + (pc & 1) * 8);
    return (unsigned)(((long)k * ld + col) * 2);
  }
}

// MFMA operand fragment (16 positions x 32 k): lane l holds X(p0 + (l & 15), 32 ks + 8 (l >> 4) + j)
template <bool T>
__device__ __forceinline__ bf16x8_t frag(const unsigned char* img, int p0, int ks, int lane) {
  const int g = lane >> 4, i16 = lane & 15;
  if constexpr (!T) {
    const int ir = p0 + i16;
    const int c = ks * 4 + g;
    return *reinterpret_cast<const bf16x8_t*>(img + ir * 128 + ((c ^ swr(ir)) << 4));
  } else {
    const int q = i16 >> 2, p = i16 & 3;
    const int k = ks * 32 + 8 * g + q;
    const int seg = (p0 >> 4) ^ swt(k);
    const int off = k * 256 + seg * 32 + p * 8;
    s4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + off));
    s4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + off + 4 * 256));
    s8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8_t, v);
  }
}

// SwiGLU-backward epilogue (down-projection data gradient): gate / up of row block i are loaded
// TWO row blocks ahead of their use, in program order before the stores of the blocks in between
// — hipcc cannot move a load above a store it cannot prove disjoint, so the plain load-compute-
// store loop serialised 8 HBM round trips per wave (the fused dgrad ran at ~1.08 PF against ~1.4
// for the plain one).  Three row blocks (48 VGPRs) are live at a time.
__device__ __forceinline__ void epi_swiglu_bwd(const f32x4_t (&acc)[8][4], unsigned short* Cb,
                                               const unsigned short* __restrict__ Gb, long ldc, long N) {
  s2_t gv[8][4], uv[8][4];
#pragma unroll
  for (int it = 0; it < 8 + 2; ++it) {
    if (it < 8) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const unsigned short* gp = Gb + (long)(16 * it) * ldc + 16 * j;
        gv[it][j] = __builtin_nontemporal_load(reinterpret_cast<const s2_t*>(gp));
        uv[it][j] = __builtin_nontemporal_load(reinterpret_cast<const s2_t*>(gp + N));
      }
    }
    if (it >= 2) {
      const int i = it - 2;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        unsigned short* p = Cb + (long)(16 * i) * ldc + 16 * j;
        const f32x4_t v = acc[i][j];
        const float gf[4] = {bf2f(gv[i][j][0] & 0xffff), bf2f(gv[i][j][0] >> 16), bf2f(gv[i][j][1] & 0xffff),
                             bf2f(gv[i][j][1] >> 16)};
        const float uf[4] = {bf2f(uv[i][j][0] & 0xffff), bf2f(uv[i][j][0] >> 16), bf2f(uv[i][j][1] & 0xffff),
                             bf2f(uv[i][j][1] >> 16)};
        float dg[4], du[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) swiglu_bwd1(v[e], gf[e], uf[e], dg[e], du[e]);
        s2_t og, ou;
        og[0] = (unsigned)f2bf(dg[0]) | ((unsigned)f2bf(dg[1]) << 16);
        og[1] = (unsigned)f2bf(dg[2]) | ((unsigned)f2bf(dg[3]) << 16);
        ou[0] = (unsigned)f2bf(du[0]) | ((unsigned)f2bf(du[1]) << 16);
        ou[1] = (unsigned)f2bf(du[2]) | ((unsigned)f2bf(du[3]) << 16);
        *reinterpret_cast<s2_t*>(p) = og;
        *reinterpret_cast<s2_t*>(p + N) = ou;
      }
    }
  }
}

// accumulate epilogue (bf16 C += acc): every old value loaded before the first store (64 VGPRs)
__device__ __forceinline__ void epi_acc_bf16(const f32x4_t (&acc)[8][4], unsigned short* Cb, long ldc, bool asm_st) {
  s2_t old[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) old[i][j] = *reinterpret_cast<const s2_t*>(Cb + (long)(16 * i) * ldc + 16 * j);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x4_t v = acc[i][j];
      v[0] += bf2f(old[i][j][0] & 0xffff);
      v[1] += bf2f(old[i][j][0] >> 16);
      v[2] += bf2f(old[i][j][1] & 0xffff);
      v[3] += bf2f(old[i][j][1] >> 16);
      s2_t o;
      o[0] = (unsigned)f2bf(v[0]) | ((unsigned)f2bf(v[1]) << 16);
      o[1] = (unsigned)f2bf(v[2]) | ((unsigned)f2bf(v[3]) << 16);
      unsigned short* p = Cb + (long)(16 * i) * ldc + 16 * j;
      if (asm_st) asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(p), "v"(o) : "memory");
      else *reinterpret_cast<s2_t*>(p) = o;
    }
}

// ---- side job: an HBM-bound elementwise pass riding on a compute-bound GEMM -------------------
// The down projection's data gradient used to carry the SwiGLU backward in its epilogue
// (EPI_SWIGLU_BWD).  Every CU reaches that epilogue at the same moment (uniform tiles), so the
// chip alternated between MFMA-bound main loops with idle HBM and HBM-bound epilogues (256 KB
// read + 256 KB written per tile) with idle matrix cores: the fused dgrad ran ~560 us (35 %)
// over the plain one at GPT-7B.  Now the dgrad stores plain dAct and the down projection's
// weight-gradient GEMM (independent of dgu) computes dgu = swiglu_bwd(dact, gu) on the side:
// every K-tile of every work item handles SIDE chunks of 1024 consecutive elements (2 per
// thread: one dword of dact / gate / up loaded, one dword of dgate / dup stored), so the
// elementwise traffic streams evenly under the MFMAs.  Measured at T 24576, H 4096, F 11008
// (tools/swiglu_side_bench.py): wgrad 1.71 ms alone, 1.99 ms with the side job (1.82 ms with
// every side access out of range, i.e. instruction cost only); dgrad + fused epilogue 2.10 ms
// vs plain dgrad (hipBLASLt via W^T) 1.59 ms; per layer 3.49 ms against 3.72 (epilogue form) and
// 3.60 (separate swiglu_bwd kernel).  Element ranges follow the global K-tile
// order (item base + t); range-checked buffer resources turn the elements past E (and the
// prologue's dummy ops) into zero loads and dropped stores, with no branch in the loop.
// Pipelining (P = t & 1 selects one of two register slots), all in phase
// j = 3, the one without LDS fragment reads (its wave group's read section has the most slack
// under the other group's MFMA segment; the stores in phase 0 and the loads in phase 1 measured
// 2.02 ms against 1.98 ms here):
//   tile t, j = 1:  ... A_hi(t+1), vmcnt(8 + 5 SIDE)
//   tile t, j = 3:  ... B_h0(t+2), W(t-2) [SwiGLU backward of slot P, 2 SIDE dword stores],
//                   L(t) [3 SIDE dword loads into slot P], vmcnt(6 + 5 SIDE)
// The waits retire exactly the half-tiles they did before (the side ops between are counted);
// L(t) is retired by the j = 3 wait of tile t+1 (one K-tile of latency cover) and consumed at
// j = 3 of tile t+2.  The prologue issues out-of-range dummies for W(-3) / L(-1) (same counts);
// L(KT-2) / L(KT-1) are stored after the loop.
constexpr unsigned SIDE_OOB = 0x80000000u;  // byte offset past every side buffer (E*4 < 2^31)
#ifndef SIDE_NT
#define SIDE_NT " nt"  // streamed once: non-temporal (1.986 vs 2.011 ms without the bit)
#endif
//  // byte offset past every side buffer (E*4 < 2^31)

template <bool AT, bool BT, int EPI, int GROUP, int SIDE = 0>
__global__ __launch_bounds__(NTHR, 1) void gemm64_kernel(G64Args args) {
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;

  // ---- work item: main tiles [0, n_main) through an XCD-bijective remap, then split items
  //      (tail tile u, K-range sp) in block order; tiles in grouped (GROUP tile-rows) order
  const int bid = blockIdx.x;
  int wg, sp = -1, u = 0;
  if (bid < args.n_main) {
    const int nwg = args.n_main;
    const int q = nwg / 8, rem = nwg % 8, x = bid % 8;
    wg = (x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q) + bid / 8;
  } else {
    const int i = bid - args.n_main;
    u = i / args.splits;
    sp = i - u * args.splits;
    wg = args.n_main + u;
  }
  const int per_group = GROUP * args.tiles_n;
  const int grp = wg / per_group;
  const int gsz = min(GROUP, args.tiles_m - grp * GROUP);
  const int inner = wg - grp * per_group;
  const int tm = grp * GROUP + inner % gsz;
  const int tn = inner / gsz;

  const long lda = args.lda, ldb = args.ldb;
  const unsigned short* Ab = AT ? args.a + (long)tm * TM : args.a + (long)tm * TM * lda;
  constexpr bool PAIRED_B = EPI == EPI_SWIGLU_FWD || EPI == EPI_UP_SWIGLU;  // gate + up rows per tile
  const unsigned short* Bb = PAIRED_B ? args.b + (long)tn * (TN / 2) * ldb
                             : BT ? args.b + (long)tn * TN : args.b + (long)tn * TN * ldb;
  const i32x4_t ra = make_rsrc(Ab), rb = make_rsrc(Bb);
  // EPI_SWIGLU_FWD: B_H1 image rows 128 + ip -> up row N + 128 tn + ip (N = F)
  const i32x4_t rb_hi = PAIRED_B ? make_rsrc(args.b + ((long)args.N + (long)tn * (TN / 2) - TN / 2) * ldb) : rb;
  // byte step of one K-tile in each operand
  const unsigned a_kstep = AT ? (unsigned)(TK * lda * 2) : (unsigned)(TK * 2);
  const unsigned b_kstep = BT ? (unsigned)(TK * ldb * 2) : (unsigned)(TK * 2);
  const int KT = sp < 0 ? args.K / TK : args.kt_part;
  const unsigned kt0 = sp < 0 ? 0u : (unsigned)(sp * args.kt_part);  // first K-tile of this item

  unsigned vo[4][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    vo[A_LO][i] = stage_voff<AT, A_LO>(i, tid, lda);
    vo[A_HI][i] = stage_voff<AT, A_HI>(i, tid, lda);
    vo[B_H0][i] = stage_voff<BT, B_H0>(i, tid, ldb);
    vo[B_H1][i] = stage_voff<BT, B_H1>(i, tid, ldb);
  }
  const unsigned lds0 = lds_addr(smem) + wave * 1024;

  // stream item: half-tile KIND of K-tile t (clamped: past-the-end items re-load the last tile)
  auto issue = [&](auto kind_c, int t) {
    constexpr int kind = decltype(kind_c)::value;
    const unsigned tc = kt0 + (unsigned)(t < KT ? t : KT - 1);
    const unsigned l = lds0 + (t & 1) * BUF + kind * HALF;
    if constexpr (kind <= A_HI) {
      const unsigned so = __builtin_amdgcn_readfirstlane(tc * a_kstep);
      bdma16(ra, vo[kind][0], so, l);
      bdma16(ra, vo[kind][1], so, l + 8192);
    } else {
      const unsigned so = __builtin_amdgcn_readfirstlane(tc * b_kstep);
      const i32x4_t r = kind == B_H1 ? rb_hi : rb;
      bdma16(r, vo[kind][0], so, l);
      bdma16(r, vo[kind][1], so, l + 8192);
    }
  };

  // ---- side job state (see above): per chunk the element index / column / gu row offset of this
  // thread's next pair, per slot the loaded dwords and the gu byte offsets they came from
  constexpr int SC = SIDE > 0 ? SIDE : 1;
  constexpr unsigned SCH = 1024u * SC;  // elements per K-tile per work item
  unsigned s_e[SC], s_f[SC], s_row[SC], s_og[2][SC], s_ou[2][SC], s_d[2][SC][3];
  i32x4_t rs_dact, rs_gu, rs_dgu;
  const unsigned sF = (unsigned)args.s_F;
  if constexpr (SIDE > 0) {
    rs_dact = make_rsrc_n(args.s_dact, args.s_E * 2u);
    rs_gu = make_rsrc_n(args.s_gu, args.s_E * 4u);
    rs_dgu = make_rsrc_n(args.s_dgu, args.s_E * 4u);
    const unsigned ktf = (unsigned)(args.K / TK);
    const unsigned gk0 = bid < args.n_main ? (unsigned)bid * ktf
                                           : (unsigned)args.n_main * ktf + (unsigned)(bid - args.n_main) * (unsigned)args.kt_part;
#pragma unroll
    for (int c = 0; c < SC; ++c) {
      const unsigned e = gk0 * SCH + 1024u * c + 2u * tid;
      const unsigned t = e / sF;
      s_e[c] = e;
      s_f[c] = e - t * sF;
      s_row[c] = t * 4u * sF;
      s_og[0][c] = s_ou[0][c] = s_og[1][c] = s_ou[1][c] = SIDE_OOB;
    }
  }
  // L: SIDE x (dact, gate, up) dword loads into slot S (DUMMY: out-of-range, no advance)
  auto side_load = [&](auto slot_c, auto dummy_c) {
    constexpr int S = decltype(slot_c)::value;
    constexpr bool DUMMY = decltype(dummy_c)::value;
#pragma unroll
    for (int c = 0; c < SC; ++c) {
      const bool ok = !DUMMY && s_e[c] < args.s_E;
      const unsigned oa = ok ? 2u * s_e[c] : SIDE_OOB;
      const unsigned og = ok ? s_row[c] + 2u * s_f[c] : SIDE_OOB;
      const unsigned ou = ok ? og + 2u * sF : SIDE_OOB;
      const i32x4_t ra_ = rs_dact, rg_ = rs_gu;
      asm volatile("buffer_load_dword %0, %1, %2, 0 offen" SIDE_NT : "=v"(s_d[S][c][0]) : "v"(oa), "s"(ra_) : "memory");
      asm volatile("buffer_load_dword %0, %1, %2, 0 offen" SIDE_NT : "=v"(s_d[S][c][1]) : "v"(og), "s"(rg_) : "memory");
      asm volatile("buffer_load_dword %0, %1, %2, 0 offen" SIDE_NT : "=v"(s_d[S][c][2]) : "v"(ou), "s"(rg_) : "memory");
      s_og[S][c] = og;
      s_ou[S][c] = ou;
      if constexpr (!DUMMY) {
        s_e[c] += SCH;
        s_f[c] += SCH;
        const bool wrap = s_f[c] >= sF;
        s_f[c] -= wrap ? sF : 0u;
        s_row[c] += wrap ? 4u * sF : 0u;
      }
    }
  };
  // W: SwiGLU backward of slot S's pairs, 2 x SIDE dword stores into dgu
  auto side_store = [&](auto slot_c) {
    constexpr int S = decltype(slot_c)::value;
#pragma unroll
    for (int c = 0; c < SC; ++c) {
      // the loads were retired by an explicit vmcnt wait; keep every use of their registers after it
      asm volatile("" : "+v"(s_d[S][c][0]), "+v"(s_d[S][c][1]), "+v"(s_d[S][c][2]));
      const unsigned d = s_d[S][c][0], gg = s_d[S][c][1], uu = s_d[S][c][2];
      float dg0, du0, dg1, du1;
      swiglu_bwd1_fast(bf2f(d & 0xffff), bf2f(gg & 0xffff), bf2f(uu & 0xffff), dg0, du0);
      swiglu_bwd1_fast(bf2f(d >> 16), bf2f(gg >> 16), bf2f(uu >> 16), dg1, du1);
      const unsigned pg = (unsigned)f2bf(dg0) | ((unsigned)f2bf(dg1) << 16);
      const unsigned pu = (unsigned)f2bf(du0) | ((unsigned)f2bf(du1) << 16);
      const unsigned og = s_og[S][c], ou = s_ou[S][c];
      const i32x4_t r = rs_dgu;
      asm volatile("buffer_store_dword %0, %1, %2, 0 offen" SIDE_NT ::"v"(pg), "v"(og), "s"(r) : "memory");
      asm volatile("buffer_store_dword %0, %1, %2, 0 offen" SIDE_NT ::"v"(pu), "v"(ou), "s"(r) : "memory");
    }
  };

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // prologue: the stream up to B_h0(1) in flight; retire A_lo/B_h0/B_h1 of K-tile 0
  issue(K_<A_LO>{}, 0);
  issue(K_<B_H0>{}, 0);
  issue(K_<B_H1>{}, 0);
  issue(K_<A_HI>{}, 0);
  issue(K_<A_LO>{}, 1);
  issue(K_<B_H0>{}, 1);
  if constexpr (SIDE > 0) {  // W(-3), L(-1): out-of-range dummies that keep the loop's counts
    side_store(K_<1>{});
    side_load(K_<1>{}, std::true_type{});
  }
  wait_vm<6 + 5 * SIDE>();
  bar();
  if (wr == 1) bar();  // wave group 1 runs one barrier behind group 0

  const int ap = wr * 64;              // this wave's first image row/col in an A half-tile
  const int bh = (wc >> 1) * HALF;     // this wave's B half-tile
  const int bp = (wc & 1) * 64;        // ... and its first position in it
  // B fragment slot j -> (half-tile byte offset, first image position): plain 16-column blocks, or
  // the paired maps of the fused epilogues (slot j + 2 holds the partner columns of slot j)
  auto bhalf = [&](int j) { return EPI == EPI_UP_SWIGLU ? (j >> 1) * HALF : bh; };
  auto bpos = [&](int j) {
    if constexpr (EPI == EPI_ROPE_QKV) return (wc & 1) * 32 + (j & 1) * 16 + (j >> 1) * 64;
    else if constexpr (EPI == EPI_UP_SWIGLU) return wc * 32 + (j & 1) * 16;
    else return bp + 16 * j;
  };
  bf16x8_t af[4][2], bfr[4][2];

  // Schedule (A/B'd by tools/gemm64_bench.py against the retired alternatives): each phase's DMA
  // is issued in the read section (before the wait and the first barrier, where the wave would
  // otherwise idle at the barrier), not right before the MFMAs, and the MFMA cluster runs under
  // s_setprio 1.  (A two-phase schedule with 32-MFMA segments measured neutral, +-1 %:
  // profiles/gemm_ld_probe_r3.txt.)
  auto mfma_quadrant = [&](auto m0_c, auto n0_c) {
    constexpr int m0 = decltype(m0_c)::value, n0 = decltype(n0_c)::value;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) acc[m0 + i][n0 + j] = mfma16(bfr[n0 + j][ks], af[i][ks], acc[m0 + i][n0 + j]);
    __builtin_amdgcn_s_setprio(0);
  };

  // each issue goes ahead of its phase's wait: the waits count 2 more pieces
  auto ktile = [&](int t, const unsigned char* buf, auto slot_c) {
    // j = 0
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) af[i][ks] = frag<AT>(buf + A_LO * HALF, ap + 16 * i, ks, lane);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) bfr[j][ks] = frag<BT>(buf + B_H0 * HALF + bhalf(j), bpos(j), ks, lane);
    issue(K_<B_H1>{}, t + 1);
    bar();
    mfma_quadrant(K_<0>{}, K_<0>{});
    bar();
    // j = 1
#pragma unroll
    for (int j = 2; j < 4; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) bfr[j][ks] = frag<BT>(buf + B_H0 * HALF + bhalf(j), bpos(j), ks, lane);
    issue(K_<A_HI>{}, t + 1);
    wait_vm<8 + 5 * SIDE>();
    bar();
    mfma_quadrant(K_<0>{}, K_<2>{});
    bar();
    // j = 2
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) af[i][ks] = frag<AT>(buf + A_HI * HALF, ap + 16 * i, ks, lane);
    issue(K_<A_LO>{}, t + 2);
    bar();
    mfma_quadrant(K_<4>{}, K_<2>{});
    bar();
    // j = 3
    issue(K_<B_H0>{}, t + 2);
    if constexpr (SIDE > 0) {
      side_store(slot_c);                     // W(t-2)
      side_load(slot_c, std::false_type{});  // L(t)
    }
    wait_vm<6 + 5 * SIDE>();
    bar();
    mfma_quadrant(K_<4>{}, K_<0>{});
    bar();
  };

  for (int t = 0; t < KT; t += 2) {
    ktile(t, smem, K_<0>{});
    ktile(t + 1, smem + BUF, K_<1>{});
  }
  if (wr == 0) bar();  // re-align the barrier count of the two groups
  wait_vm<0>();        // the clamped tail items are still landing
  if constexpr (SIDE > 0) {  // W(KT-2), W(KT-1)
    side_store(K_<0>{});
    side_store(K_<1>{});
  }

  // ---- epilogue: lane holds C[m = .. + (l&15)][n = .. + 4(l>>4) + r], r = 0..3
  const int g = lane >> 4, i16 = lane & 15;
  if constexpr (EPI == EPI_ROPE_QKV) {
    // slot j (j = 0, 1) holds dims d = (wc & 1) * 32 + 16 j + 4 g + r of head h, slot j + 2 dims d + 64
    const int h = 2 * tn + (wc >> 1);
    const int nrot = args.nq + args.nkv;  // heads [0, nrot) rotate
    unsigned short* dst0;
    long dst_ld;
    if (h < args.nq) {
      dst0 = args.c + (long)h * 128;
      dst_ld = (long)args.nq * 128;
    } else if (h < nrot) {
      dst0 = args.out2 + (long)(h - args.nq) * 128;
      dst_ld = (long)args.nkv * 128;
    } else {
      dst0 = args.out3 + (long)(h - nrot) * 128;
      dst_ld = (long)args.nkv * 128;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int t = tm * TM + wr * 128 + 16 * i + i16;
      unsigned short* drow = dst0 + (long)t * dst_ld;
      const long p = args.pos ? (long)args.pos[t] : (long)(t % args.seq);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int d = (wc & 1) * 32 + 16 * j + 4 * g;
        float o1[4], o2[4];
        if (h < nrot) {  // as rope_fwd_kernel on the bf16-stored projection
          const f32x4_t cs = *reinterpret_cast<const f32x4_t*>(args.cosT + p * 64 + d);
          const f32x4_t sn = *reinterpret_cast<const f32x4_t*>(args.sinT + p * 64 + d);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float a = bf2f(f2bf(acc[i][j][e])), b = bf2f(f2bf(acc[i][j + 2][e]));
            o1[e] = a * cs[e] - b * sn[e];
            o2[e] = b * cs[e] + a * sn[e];
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            o1[e] = acc[i][j][e];
            o2[e] = acc[i][j + 2][e];
          }
        }
        s2_t a1, a2;
        a1[0] = (unsigned)f2bf(o1[0]) | ((unsigned)f2bf(o1[1]) << 16);
        a1[1] = (unsigned)f2bf(o1[2]) | ((unsigned)f2bf(o1[3]) << 16);
        a2[0] = (unsigned)f2bf(o2[0]) | ((unsigned)f2bf(o2[1]) << 16);
        a2[1] = (unsigned)f2bf(o2[2]) | ((unsigned)f2bf(o2[3]) << 16);
        *reinterpret_cast<s2_t*>(drow + d) = a1;
        *reinterpret_cast<s2_t*>(drow + 64 + d) = a2;
      }
    }
    return;
  }
  if constexpr (EPI == EPI_UP_SWIGLU) {
    // slot j (j = 0, 1): gate cols 128 tn + wc * 32 + 16 j + 4 g + r; slot j + 2: the same up cols
    const long F = args.N;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const long t = (long)tm * TM + wr * 128 + 16 * i + i16;
      unsigned short* gurow = args.c + t * args.ldc;
      unsigned short* arow = args.out2 + t * F;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = tn * 128 + wc * 32 + 16 * j + 4 * g;
        float o[4];
        s2_t pg, pu, pa;
        unsigned short gb[4], ub[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {  // as swiglu_fwd_kernel on the bf16-stored g / u
          gb[e] = f2bf(acc[i][j][e]);
          ub[e] = f2bf(acc[i][j + 2][e]);
          const float gg = bf2f(gb[e]), uu = bf2f(ub[e]);
          o[e] = gg * (1.f / (1.f + __expf(-gg))) * uu;
        }
        pg[0] = (unsigned)gb[0] | ((unsigned)gb[1] << 16);
        pg[1] = (unsigned)gb[2] | ((unsigned)gb[3] << 16);
        pu[0] = (unsigned)ub[0] | ((unsigned)ub[1] << 16);
        pu[1] = (unsigned)ub[2] | ((unsigned)ub[3] << 16);
        pa[0] = (unsigned)f2bf(o[0]) | ((unsigned)f2bf(o[1]) << 16);
        pa[1] = (unsigned)f2bf(o[2]) | ((unsigned)f2bf(o[3]) << 16);
        *reinterpret_cast<s2_t*>(gurow + col) = pg;
        *reinterpret_cast<s2_t*>(gurow + F + col) = pu;
        *reinterpret_cast<s2_t*>(arow + col) = pa;
      }
    }
    return;
  }
  if constexpr (EPI == EPI_SWIGLU_FWD) {
    if (sp >= 0) {  // split item (uniform per workgroup): the generic partial tile, gate cols [0, 128), up 128 +
      float* W = args.ws + ((long)u * args.splits + sp) * (TM * TN) + (wr * 128 + i16) * TN + wc * 64 + 4 * g;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) *reinterpret_cast<f32x4_t*>(W + (16 * i) * TN + 16 * j) = acc[i][j];
      return;
    }
    // up waves (wc 2, 3) hand their tiles to the gate waves (wc 0, 1) with the same (wr, i, j, lane)
    // through the now idle 128-KB LDS image: [wr][wc & 1][i][j][lane] f32x4
    __syncthreads();
    f32x4_t* xch = reinterpret_cast<f32x4_t*>(smem) + (wr * 2 + (wc & 1)) * (8 * 4 * 64) + lane;
    if (wc >= 2) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) xch[(i * 4 + j) * 64] = acc[i][j];
    }
    __syncthreads();
    if (wc >= 2) return;
    unsigned short* Ab2 = args.c + (long)(tm * TM + wr * 128 + i16) * args.ldc + tn * (TN / 2) + wc * 64 + 4 * g;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4_t gv = acc[i][j], uv = xch[(i * 4 + j) * 64];
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {  // as swiglu_fwd_kernel on the bf16-stored g / u
          const float gg = bf2f(f2bf(gv[e])), uu = bf2f(f2bf(uv[e]));
          o[e] = gg * (1.f / (1.f + __expf(-gg))) * uu;
        }
        s2_t pk;
        pk[0] = (unsigned)f2bf(o[0]) | ((unsigned)f2bf(o[1]) << 16);
        pk[1] = (unsigned)f2bf(o[2]) | ((unsigned)f2bf(o[3]) << 16);
        *reinterpret_cast<s2_t*>(Ab2 + (long)(16 * i) * args.ldc + 16 * j) = pk;
      }
    return;
  }
  if (sp >= 0) {  // split item: fp32 partial tile, row-major 256 x 256
    float* W = args.ws + ((long)u * args.splits + sp) * (TM * TN) + (wr * 128 + i16) * TN + wc * 64 + 4 * g;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) *reinterpret_cast<f32x4_t*>(W + (16 * i) * TN + 16 * j) = acc[i][j];
    return;
  }
  if constexpr (epi_f32(EPI)) {
    float* Cf = reinterpret_cast<float*>(args.c) + (long)(tm * TM + wr * 128 + i16) * args.ldc + tn * TN + wc * 64 + 4 * g;
    if constexpr (EPI == EPI_ACC_F32) {  // olds of a half (16 x 16 B) loaded before its stores
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        f32x4_t old[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            old[i][j] = *reinterpret_cast<const f32x4_t*>(Cf + (long)(16 * (4 * hf + i)) * args.ldc + 16 * j);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            *reinterpret_cast<f32x4_t*>(Cf + (long)(16 * (4 * hf + i)) * args.ldc + 16 * j) = old[i][j] + acc[4 * hf + i][j];
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) *reinterpret_cast<f32x4_t*>(Cf + (long)(16 * i) * args.ldc + 16 * j) = acc[i][j];
    return;
  }
  unsigned short* Cb = args.c + (long)(tm * TM + wr * 128 + i16) * args.ldc + tn * TN + wc * 64 + 4 * g;
  if constexpr (EPI == EPI_SWIGLU_BWD) {
    epi_swiglu_bwd(acc, Cb, args.aux + (Cb - args.c), args.ldc, args.N);
    return;
  }
  if constexpr (EPI == EPI_ACC) {
    epi_acc_bf16(acc, Cb, args.ldc, false);
    return;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      unsigned short* p = Cb + (long)(16 * i) * args.ldc + 16 * j;
      f32x4_t v = acc[i][j];
      s2_t o;
      o[0] = (unsigned)f2bf(v[0]) | ((unsigned)f2bf(v[1]) << 16);
      o[1] = (unsigned)f2bf(v[2]) | ((unsigned)f2bf(v[3]) << 16);
      *reinterpret_cast<s2_t*>(p) = o;
    }
  }
}


// ---- 4-wave kernel (config variants >= 4): one 128x128 output block per wave ---------------------
// The 8-wave kernel above reads (128 + 64) x 64 operand elements from LDS per wave per K-tile for
// a 128x64 block: 192 KB of ds_read per CU per K-tile, 75 % of the MFMA time of the tile at the
// LDS's 256 B/clk.  hipBLASLt's MT256x256x64 kernel (rocprof: 256 threads, 130 KB LDS, 252 VGPRs)
// gives each of 4 waves a 128x128 block instead: (128 + 128) x 64 per wave, 128 KB per CU per
// K-tile (-33 % LDS traffic per FLOP; a ds_read costs power the MFMA clock pays for).  Same
// staging as above (half-tile images, LDS-DMA, swizzles, clamped tail items, XCD remap, split
// tail); what changes:
//   * waves (wr, wc) = (wave >> 1, wave & 1): rows wr*128 + [0,128) = m-tiles 0-3 in A_lo at image
//     positions wr*64.., m-tiles 4-7 in A_hi; cols wc*128 + [0,128) = all of half-tile B_h{wc}.
//     acc[8][8] (256 fp32 per lane) lives in the accumulation registers (one wave per SIMD).
//   * one wave per SIMD means no ping-pong partner: each phase's MFMAs run on fragments read in
//     the PREVIOUS phase, while this phase's ds_reads (for the next) and DMA issue go out under
//     them.  Phase plan of K-tile t (buffer t & 1), 32 MFMAs each, one barrier at the end:
//        P0  MFMA (m0-3, n0-3) [a_lo, b03]   read b47   <- B(t)      issue A_lo(t+2)  vmcnt(20)
//        P1  MFMA (m0-3, n4-7) [a_lo, b47]   read a_hi  <- A_hi(t)   issue B_h0(t+2)  vmcnt(20)
//        P2  MFMA (m4-7, n4-7) [a_hi, b47]   read a_lo  <- A_lo(t+1) issue B_h1(t+2)  vmcnt(16)
//        P3  MFMA (m4-7, n0-3) [a_hi, b03]   read b03'  <- B(t+1)    issue A_hi(t+2)  -
//     b03 is double-buffered by K-tile parity (it is read for t+1 while t's is still in use).
//     RAW: each phase ends with vmcnt(N) retiring exactly the half-tile the next phase reads, then
//     lgkmcnt(0) + s_barrier.  WAR: every DMA goes into a slot whose last ds_reads were issued at
//     least one phase earlier (so retired before that phase's closing barrier).  The waits keep 4-5
//     half-tiles (16-20 DMA instructions per thread) in flight.
constexpr int NT4 = 256;
// two MFMAs (acc row i x n-tiles j, j+1, one K-slice) / the same with one LDS-DMA piece between
// them (M0 written ahead of the first MFMA, so the MFMA covers the M0 -> LDS-DMA wait state): the
// K-loop's statements, so each fragment read and each DMA piece gets an MFMA gap of its own.
// Accumulators are pinned to the accumulation registers ("+a"; hipcc's own MFMA selection moved
// them through VGPRs and spilled: 256 accumulators + 160 fragment registers exceed the 256
// VGPRs); the "memory" clobber pins the reads / DMA issues placed between two statements to their
// gap.  Hazards (guide §5.7 item 2): MFMA -> MFMA accumulate chains need no wait states; the
// epilogue's reads are fenced after the loop (g4w_fence).
__device__ __forceinline__ void g4w_pair(f32x4_t& c0, f32x4_t& c1, const bf16x8_t& a, const bf16x8_t& b0,
                                         const bf16x8_t& b1) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %3, %2, %0\n\t"
               "v_mfma_f32_16x16x32_bf16 %1, %4, %2, %1"
               : "+a"(c0), "+a"(c1)
               : "v"(a), "v"(b0), "v"(b1)
               : "memory");
}
// the same with C = 0 (an item's first K-slice): the accumulators are defined here, not carried
// from a zeroing through the item loop's back-edge (persistent kernel)
__device__ __forceinline__ void g4w_pair_z(f32x4_t& c0, f32x4_t& c1, const bf16x8_t& a, const bf16x8_t& b0,
                                           const bf16x8_t& b1) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %3, %2, 0\n\t"
               "v_mfma_f32_16x16x32_bf16 %1, %4, %2, 0"
               : "=a"(c0), "=a"(c1)
               : "v"(a), "v"(b0), "v"(b1)
               : "memory");
}
__device__ __forceinline__ void g4w_pair_dma(f32x4_t& c0, f32x4_t& c1, const bf16x8_t& a, const bf16x8_t& b0,
                                             const bf16x8_t& b1, unsigned voff, i32x4_t rsrc, unsigned soff,
                                             unsigned lds_byte) {
  asm volatile("s_mov_b32 m0, %8\n\t"
               "v_mfma_f32_16x16x32_bf16 %0, %3, %2, %0\n\t"
               "buffer_load_dwordx4 %5, %6, %7 offen lds\n\t"
               "v_mfma_f32_16x16x32_bf16 %1, %4, %2, %1"
               : "+a"(c0), "+a"(c1)
               : "v"(a), "v"(b0), "v"(b1), "v"(voff), "s"(rsrc), "s"(soff), "s"(lds_byte)
               : "memory");
}

__device__ __forceinline__ void g4w_fence(f32x4_t (&acc)[8][8]) {
  asm volatile("s_nop 7\n\ts_nop 7"
               : "+a"(acc[4][0]), "+a"(acc[4][1]), "+a"(acc[4][2]), "+a"(acc[4][3]), "+a"(acc[5][0]), "+a"(acc[5][1]),
                 "+a"(acc[5][2]), "+a"(acc[5][3]), "+a"(acc[6][0]), "+a"(acc[6][1]), "+a"(acc[6][2]), "+a"(acc[6][3]),
                 "+a"(acc[7][0]), "+a"(acc[7][1]), "+a"(acc[7][2]), "+a"(acc[7][3]));
}

// the 2-phase kernel's last phase writes every accumulator; its last 16 MFMAs are rows 6 and 7
__device__ __forceinline__ void g2p_fence(f32x4_t (&acc)[8][8]) {
  asm volatile("s_nop 7\n\ts_nop 7"
               : "+a"(acc[6][0]), "+a"(acc[6][1]), "+a"(acc[6][2]), "+a"(acc[6][3]), "+a"(acc[6][4]), "+a"(acc[6][5]),
                 "+a"(acc[6][6]), "+a"(acc[6][7]), "+a"(acc[7][0]), "+a"(acc[7][1]), "+a"(acc[7][2]), "+a"(acc[7][3]),
                 "+a"(acc[7][4]), "+a"(acc[7][5]), "+a"(acc[7][6]), "+a"(acc[7][7]));
}

// 4-wave epilogues (lane holds C[wr*128 + 16 i + (l & 15)][wc*128 + 16 j + 4 (l >> 4) + r]): split
// partial, fp32 store / accumulate, bf16 store / accumulate, fused RoPE-QKV / SwiGLU forward
template <int EPI, bool RS = false>
__device__ __forceinline__ void g4w_epilogue(const G64Args& args, f32x4_t (&acc)[8][8], int tm, int tn, int wr, int wc,
                                             int lane, int sp, int u, const float* rsl = nullptr) {
  constexpr bool PAIRED_B = EPI == EPI_UP_SWIGLU || EPI == EPI_SWIGLU_FWD;
  const int g = lane >> 4, i16 = lane & 15;
  // RS: the lane's row 16 i + i16 of the wave's 128 is scaled by rs[row], read per row block from
  // the tile's 256 rs values staged in LDS (rsl; split partials stay unscaled: gemm64_split_reduce
  // scales their sum)
  auto row_scale = [&](int i) __attribute__((always_inline)) { return RS ? rsl[wr * 128 + 16 * i + i16] : 1.f; };
  if constexpr (EPI == EPI_ROPE_QKV) {
    if (sp >= 0) {  // a split tail item: fp32 partials; gemm64_split_reduce applies the RoPE epilogue
      float* W = args.ws + ((long)u * args.splits + sp) * (TM * TN) + (wr * 128 + i16) * TN + wc * 128 + 4 * g;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) *reinterpret_cast<f32x4_t*>(W + (16 * i) * TN + 16 * j) = acc[i][j];
      return;
    }
    // a 256-column tile = 2 heads of D = 128: wave wc owns head 2 tn + wc whole; n-tile j (< 4)
    // holds dims d = 16 j + 4 g + r, n-tile j + 4 the rotation partners d + 64
    const int h = 2 * tn + wc;
    const int nrot = args.nq + args.nkv;  // heads [0, nrot) rotate
    unsigned short* dst0;
    long dst_ld;
    if (h < args.nq) {
      dst0 = args.c + (long)h * 128;
      dst_ld = (long)args.nq * 128;
    } else if (h < nrot) {
      dst0 = args.out2 + (long)(h - args.nq) * 128;
      dst_ld = (long)args.nkv * 128;
    } else {
      dst0 = args.out3 + (long)(h - nrot) * 128;
      dst_ld = (long)args.nkv * 128;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int t = tm * TM + wr * 128 + 16 * i + i16;
      unsigned short* drow = dst0 + (long)t * dst_ld;
      const long p = args.pos ? (long)args.pos[t] : (long)(t % args.seq);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int d = 16 * j + 4 * g;
        float o1[4], o2[4];
        if (h < nrot) {  // as rope_fwd_kernel on the bf16-stored projection
          const f32x4_t cs = *reinterpret_cast<const f32x4_t*>(args.cosT + p * 64 + d);
          const f32x4_t sn = *reinterpret_cast<const f32x4_t*>(args.sinT + p * 64 + d);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float a = bf2f(f2bf(acc[i][j][e])), b = bf2f(f2bf(acc[i][j + 4][e]));
            o1[e] = a * cs[e] - b * sn[e];
            o2[e] = b * cs[e] + a * sn[e];
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            o1[e] = acc[i][j][e];
            o2[e] = acc[i][j + 4][e];
          }
        }
        s2_t a1, a2;
        a1[0] = (unsigned)f2bf(o1[0]) | ((unsigned)f2bf(o1[1]) << 16);
        a1[1] = (unsigned)f2bf(o1[2]) | ((unsigned)f2bf(o1[3]) << 16);
        a2[0] = (unsigned)f2bf(o2[0]) | ((unsigned)f2bf(o2[1]) << 16);
        a2[1] = (unsigned)f2bf(o2[2]) | ((unsigned)f2bf(o2[3]) << 16);
        *reinterpret_cast<s2_t*>(drow + d) = a1;
        *reinterpret_cast<s2_t*>(drow + 64 + d) = a2;
      }
    }
    return;
  }
  if constexpr (PAIRED_B) {
    if constexpr (EPI == EPI_SWIGLU_FWD) {
      if (sp >= 0) {  // a split tail item: fp32 partials, gate cols at [0, 128) and up cols at 128 + [0, 128)
        // of the workspace tile; gemm64_split_reduce applies the row scale and the SwiGLU
        float* W = args.ws + ((long)u * args.splits + sp) * (TM * TN) + (wr * 128 + i16) * TN + wc * 64 + 4 * g;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 8; ++j)
            *reinterpret_cast<f32x4_t*>(W + (16 * i) * TN + (j < 4 ? 16 * j : 128 + 16 * (j - 4))) = acc[i][j];
        return;
      }
    }
    // n-tile j (< 4): gate cols 128 tn + wc * 64 + 16 j + 4 g + r; n-tile j + 4: the same up cols.
    // EPI_UP_SWIGLU stores gu [T, 2F] and act [T, F]; EPI_SWIGLU_FWD only act (into C, ldc = F)
    const long F = args.N;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const long t = (long)tm * TM + wr * 128 + 16 * i + i16;
      const float ri = row_scale(i);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = tn * 128 + wc * 64 + 16 * j + 4 * g;
        float o[4];
        unsigned short gb[4], ub[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {  // as swiglu_fwd_kernel on the bf16-stored g / u
          gb[e] = f2bf(RS ? acc[i][j][e] * ri : acc[i][j][e]);
          ub[e] = f2bf(RS ? acc[i][j + 4][e] * ri : acc[i][j + 4][e]);
          const float gg = bf2f(gb[e]), uu = bf2f(ub[e]);
          o[e] = gg * (1.f / (1.f + __expf(-gg))) * uu;
        }
        s2_t pa;
        pa[0] = (unsigned)f2bf(o[0]) | ((unsigned)f2bf(o[1]) << 16);
        pa[1] = (unsigned)f2bf(o[2]) | ((unsigned)f2bf(o[3]) << 16);
        if constexpr (EPI == EPI_UP_SWIGLU) {
          s2_t pg, pu;
          pg[0] = (unsigned)gb[0] | ((unsigned)gb[1] << 16);
          pg[1] = (unsigned)gb[2] | ((unsigned)gb[3] << 16);
          pu[0] = (unsigned)ub[0] | ((unsigned)ub[1] << 16);
          pu[1] = (unsigned)ub[2] | ((unsigned)ub[3] << 16);
          unsigned short* gurow = args.c + t * args.ldc;
          *reinterpret_cast<s2_t*>(gurow + col) = pg;
          *reinterpret_cast<s2_t*>(gurow + F + col) = pu;
          *reinterpret_cast<s2_t*>(args.out2 + t * F + col) = pa;
        } else {
          *reinterpret_cast<s2_t*>(args.c + t * args.ldc + col) = pa;
        }
      }
    }
    return;
  }
  if (sp >= 0) {
    float* W = args.ws + ((long)u * args.splits + sp) * (TM * TN) + (wr * 128 + i16) * TN + wc * 128 + 4 * g;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) *reinterpret_cast<f32x4_t*>(W + (16 * i) * TN + 16 * j) = acc[i][j];
    return;
  }
  if constexpr (epi_f32(EPI)) {
    float* Cf = reinterpret_cast<float*>(args.c) + (long)(tm * TM + wr * 128 + i16) * args.ldc + tn * TN + wc * 128 + 4 * g;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (EPI == EPI_ACC_F32) {
        f32x4_t old[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) old[j] = *reinterpret_cast<const f32x4_t*>(Cf + (long)(16 * i) * args.ldc + 16 * j);
#pragma unroll
        for (int j = 0; j < 8; ++j) *reinterpret_cast<f32x4_t*>(Cf + (long)(16 * i) * args.ldc + 16 * j) = old[j] + acc[i][j];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) *reinterpret_cast<f32x4_t*>(Cf + (long)(16 * i) * args.ldc + 16 * j) = acc[i][j];
      }
    }
    return;
  }
  // bf16: 16-byte stores.  v_permlane16_swap pairs n-tiles j, j + 1 (j even): lane row-group g
  // then holds 8 consecutive columns 16 (j + (g & 1)) + 8 (g >> 1) + [0, 8) of its row, so a
  // row's 4 lanes write 64 contiguous bytes per instruction and a thread issues 32 stores (not 64
  // of 8 bytes) -- half the vector-memory operations the persistent kernel's counted waits after an
  // epilogue must allow for
  const int cs = 16 * (g & 1) + 8 * (g >> 1);
  unsigned short* Cb = args.c + (long)(tm * TM + wr * 128 + i16) * args.ldc + tn * TN + wc * 128 + cs;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint4 old[4];
    const float ri = row_scale(i);
    if constexpr (EPI == EPI_ACC) {
#pragma unroll
      for (int jp = 0; jp < 4; ++jp) old[jp] = *reinterpret_cast<const uint4*>(Cb + (long)(16 * i) * args.ldc + 32 * jp);
    }
#pragma unroll
    for (int jp = 0; jp < 4; ++jp) {
      const int j = 2 * jp;
      uint4 o;
      if constexpr (EPI == EPI_ACC) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][j][e]), __float_as_uint(acc[i][j + 1][e]),
                                                          false, false);
          v[e] = __uint_as_float(r[0]);
          v[4 + e] = __uint_as_float(r[1]);
        }
        const unsigned ow[4] = {old[jp].x, old[jp].y, old[jp].z, old[jp].w};
        unsigned pk[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          pk[e] = (unsigned)f2bf(v[2 * e] + bf2f(ow[e] & 0xffff)) | ((unsigned)f2bf(v[2 * e + 1] + bf2f(ow[e] >> 16)) << 16);
        o = make_uint4(pk[0], pk[1], pk[2], pk[3]);
      } else {
        f32x4_t c0 = acc[i][j], c1 = acc[i][j + 1];
        if constexpr (RS) {
          c0 *= ri;
          c1 *= ri;
        }
        const unsigned x0 = (unsigned)f2bf(c0[0]) | ((unsigned)f2bf(c0[1]) << 16);
        const unsigned x1 = (unsigned)f2bf(c0[2]) | ((unsigned)f2bf(c0[3]) << 16);
        const unsigned y0 = (unsigned)f2bf(c1[0]) | ((unsigned)f2bf(c1[1]) << 16);
        const unsigned y1 = (unsigned)f2bf(c1[2]) | ((unsigned)f2bf(c1[3]) << 16);
        const auto r0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
        const auto r1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
        o = make_uint4(r0[0], r1[0], r0[1], r1[1]);
      }
      *reinterpret_cast<uint4*>(Cb + (long)(16 * i) * args.ldc + 32 * jp) = o;
    }
    __builtin_amdgcn_sched_barrier(0);  // one row's conversions live at a time (no spills)
  }
}

// Side job (SIDE > 0: the down projection's wgrad computing dgu = swiglu_bwd(dact, gu), as in the
// 8-wave kernel above): SIDE chunks of 1024 elements per K-tile per work item, each thread two
// element pairs per chunk (256 threads).  Phase P3 of K-tile t, after its DMA, stores W(t-2)
// (slot t & 1) and loads L(t) into the same slot: S_OPS = 10 SIDE vector-memory ops that the
// waits count past (P0: 20 + 2 S_OPS, P1: 20 + S_OPS, P2: 16 + S_OPS); L(t) is retired by the P1
// wait of K-tile t+2, before W(t) at P3 of K-tile t+2.  The prologue issues out-of-range dummies
// W/L(-2) and W/L(-1) at their stream positions so every count holds from the first phase.
// Each phase: 16 statements of 2 MFMAs, the next phase's fragment reads in the first half, the
// phase's 4 DMA pieces inside the second (retired orderings: profiles/ab_gemm64_config_r4.log)
template <bool AT, bool BT, int EPI, int GROUP, int SIDE = 0>
__global__ __launch_bounds__(NT4, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm4w_kernel(G64Args args) {
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;

  const int bid = blockIdx.x;
  int wg, sp = -1, u = 0;
  if (bid < args.n_main) {
    const int nwg = args.n_main;
    const int q = nwg / 8, rem = nwg % 8, x = bid % 8;
    wg = (x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q) + bid / 8;
  } else {
    const int i = bid - args.n_main;
    u = i / args.splits;
    sp = i - u * args.splits;
    wg = args.n_main + u;
  }
  const int per_group = GROUP * args.tiles_n;
  const int grp = wg / per_group;
  const int gsz = min(GROUP, args.tiles_m - grp * GROUP);
  const int inner = wg - grp * per_group;
  const int tm = grp * GROUP + inner % gsz;
  const int tn = inner / gsz;

  const long lda = args.lda, ldb = args.ldb;
  const int tml = (args.probe & 8) ? 0 : tm, tnl = (args.probe & 8) ? 0 : tn;  // probe 8: one tile's operands
  const unsigned short* Ab = AT ? args.a + (long)tml * TM : args.a + (long)tml * TM * lda;
  constexpr bool PAIRED_B = EPI == EPI_UP_SWIGLU || EPI == EPI_SWIGLU_FWD;  // gate + up rows per tile
  const unsigned short* Bb = PAIRED_B ? args.b + (long)tnl * (TN / 2) * ldb
                             : BT ? args.b + (long)tnl * TN : args.b + (long)tnl * TN * ldb;
  i32x4_t ra = make_rsrc(Ab), rb = make_rsrc(Bb);
  // paired: B_H1 image rows 128 + ip -> up row N + 128 tn + ip (N = F)
  i32x4_t rb_hi = PAIRED_B ? make_rsrc(args.b + ((long)args.N + (long)tnl * (TN / 2) - TN / 2) * ldb) : rb;
  if (args.probe & 1) ra[2] = rb[2] = rb_hi[2] = 0;
  if (args.probe & 32) ra[2] = 0;            // probe 32: A loads out of range only
  if (args.probe & 64) rb[2] = rb_hi[2] = 0;  // probe 64: B loads out of range only
  // probe 16: every K-tile re-reads K-tile 0 (a 64 KB working set per tile: L2-hit latency only)
  const unsigned a_kstep = (args.probe & 16) ? 0u : AT ? (unsigned)(TK * lda * 2) : (unsigned)(TK * 2);
  const unsigned b_kstep = (args.probe & 16) ? 0u : BT ? (unsigned)(TK * ldb * 2) : (unsigned)(TK * 2);
  const int KT = sp < 0 ? args.K / TK : args.kt_part;
  const unsigned kt0 = sp < 0 ? 0u : (unsigned)(sp * args.kt_part);

  unsigned vo[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    vo[A_LO][i] = stage_voff<AT, A_LO, NT4>(i, tid, lda);
    vo[A_HI][i] = stage_voff<AT, A_HI, NT4>(i, tid, lda);
    vo[B_H0][i] = stage_voff<BT, B_H0, NT4>(i, tid, ldb);
    vo[B_H1][i] = stage_voff<BT, B_H1, NT4>(i, tid, ldb);
  }
  const unsigned lds0 = lds_addr(smem) + wave * 1024;
  auto issue = [&](auto kind_c, int t) {
    constexpr int kind = decltype(kind_c)::value;
    const unsigned tc = kt0 + (unsigned)(t < KT ? t : KT - 1);
    const unsigned l = lds0 + (t & 1) * BUF + kind * HALF;
    const unsigned so = __builtin_amdgcn_readfirstlane(tc * (kind <= A_HI ? a_kstep : b_kstep));
    const i32x4_t r = kind <= A_HI ? ra : kind == B_H1 ? rb_hi : rb;
#pragma unroll
    for (int i = 0; i < 4; ++i) bdma16(r, vo[kind][i], so, l + i * 4096);
  };

  // ---- side job state: per sub-chunk (2 per chunk) the element index / column / gu row offset
  // of this thread's next pair, per slot the loaded dwords and the gu byte offsets they came from
  constexpr int SC = SIDE > 0 ? 2 * SIDE : 1;
  constexpr unsigned SCH = 1024u * (SIDE > 0 ? SIDE : 1);  // elements per K-tile per work item
  constexpr int S_OPS = 10 * SIDE;
  unsigned s_e[SC], s_f[SC], s_row[SC], s_og[2][SC], s_ou[2][SC], s_d[2][SC][3];
  i32x4_t rs_dact, rs_gu, rs_dgu;
  const unsigned sF = (unsigned)args.s_F;
  if constexpr (SIDE > 0) {
    rs_dact = make_rsrc_n(args.s_dact, args.s_E * 2u);
    rs_gu = make_rsrc_n(args.s_gu, args.s_E * 4u);
    rs_dgu = make_rsrc_n(args.s_dgu, args.s_E * 4u);
    const unsigned ktf = (unsigned)(args.K / TK);
    const unsigned gk0 = bid < args.n_main ? (unsigned)bid * ktf
                                           : (unsigned)args.n_main * ktf + (unsigned)(bid - args.n_main) * (unsigned)args.kt_part;
#pragma unroll
    for (int c = 0; c < SC; ++c) {
      const unsigned e = gk0 * SCH + 512u * c + 2u * tid;
      const unsigned t = e / sF;
      s_e[c] = e;
      s_f[c] = e - t * sF;
      s_row[c] = t * 4u * sF;
      s_og[0][c] = s_ou[0][c] = s_og[1][c] = s_ou[1][c] = SIDE_OOB;
    }
  }
  auto side_load = [&](auto slot_c, auto dummy_c) {
    constexpr int S = decltype(slot_c)::value;
    constexpr bool DUMMY = decltype(dummy_c)::value;
#pragma unroll
    for (int c = 0; c < SC; ++c) {
      const bool ok = !DUMMY && s_e[c] < args.s_E;
      const unsigned oa = ok ? 2u * s_e[c] : SIDE_OOB;
      const unsigned og = ok ? s_row[c] + 2u * s_f[c] : SIDE_OOB;
      const unsigned ou = ok ? og + 2u * sF : SIDE_OOB;
      const i32x4_t ra_ = rs_dact, rg_ = rs_gu;
      asm volatile("buffer_load_dword %0, %1, %2, 0 offen" SIDE_NT : "=v"(s_d[S][c][0]) : "v"(oa), "s"(ra_) : "memory");
      asm volatile("buffer_load_dword %0, %1, %2, 0 offen" SIDE_NT : "=v"(s_d[S][c][1]) : "v"(og), "s"(rg_) : "memory");
      asm volatile("buffer_load_dword %0, %1, %2, 0 offen" SIDE_NT : "=v"(s_d[S][c][2]) : "v"(ou), "s"(rg_) : "memory");
      s_og[S][c] = og;
      s_ou[S][c] = ou;
      if constexpr (!DUMMY) {
        s_e[c] += SCH;
        s_f[c] += SCH;
        const bool wrap = s_f[c] >= sF;  // SCH <= F (side_chunks): at most one row wrap per K-tile
        s_f[c] -= wrap ? sF : 0u;
        s_row[c] += wrap ? 4u * sF : 0u;
      }
    }
  };
  auto side_store = [&](auto slot_c) {
    constexpr int S = decltype(slot_c)::value;
#pragma unroll
    for (int c = 0; c < SC; ++c) {
      asm volatile("" : "+v"(s_d[S][c][0]), "+v"(s_d[S][c][1]), "+v"(s_d[S][c][2]));
      const unsigned d = s_d[S][c][0], gg = s_d[S][c][1], uu = s_d[S][c][2];
      float dg0, du0, dg1, du1;
      swiglu_bwd1_fast(bf2f(d & 0xffff), bf2f(gg & 0xffff), bf2f(uu & 0xffff), dg0, du0);
      swiglu_bwd1_fast(bf2f(d >> 16), bf2f(gg >> 16), bf2f(uu >> 16), dg1, du1);
      const unsigned pg = (unsigned)f2bf(dg0) | ((unsigned)f2bf(dg1) << 16);
      const unsigned pu = (unsigned)f2bf(du0) | ((unsigned)f2bf(du1) << 16);
      const unsigned og = s_og[S][c], ou = s_ou[S][c];
      const i32x4_t r = rs_dgu;
      asm volatile("buffer_store_dword %0, %1, %2, 0 offen" SIDE_NT ::"v"(pg), "v"(og), "s"(r) : "memory");
      asm volatile("buffer_store_dword %0, %1, %2, 0 offen" SIDE_NT ::"v"(pu), "v"(ou), "s"(r) : "memory");
    }
  };

  f32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int ap = wr * 64;
  // B fragments: n-tiles 0-3 (b03) and 4-7 (b47) are positions 0-63 / 64-127 of half-tile
  // B_h{wc}; paired (gate/up) tiles take this wave's 64 gate columns wc*64.. of B_h0 as b03 and
  // the matching 64 up columns of B_h1 as b47, so acc[i][j] / acc[i][j + 4] are a gate/up pair
  const int bo03 = PAIRED_B ? B_H0 * HALF : (B_H0 + wc) * HALF, p03 = PAIRED_B ? wc * 64 : 0;
  const int bo47 = PAIRED_B ? B_H1 * HALF : (B_H0 + wc) * HALF, p47 = PAIRED_B ? wc * 64 : 64;
  bf16x8_t a_lo[4][2], a_hi[4][2], b47[4][2], b03[2][4][2];
  auto rdA = [&](bf16x8_t (&d)[4][2], const unsigned char* img) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) d[i][ks] = frag<AT>(img, ap + 16 * i, ks, lane);
  };
  auto rdB = [&](bf16x8_t (&d)[4][2], const unsigned char* img, int p0) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) d[j][ks] = frag<BT>(img, p0 + 16 * j, ks, lane);
  };
  // lgkmcnt(0) through the builtin: hipcc's waitcnt pass then knows the fragment reads are done
  // (an asm wait is opaque to it, and it re-waited lgkmcnt(0) ahead of the next MFMA block --
  // after the NEXT phase's reads had been issued, serialising them)
  auto sync = [&](auto n_c) {
    constexpr int N = decltype(n_c)::value;
    if constexpr (N >= 0) wait_vm<N>();
    __builtin_amdgcn_s_waitcnt(0xC07F);  // gfx9 encoding: vmcnt 63, expcnt 7, lgkmcnt 0
    if (!(args.probe & 2)) bar();
  };

  // one phase: 16 statements of 2 MFMAs (K-slice q >> 3, row (q >> 1) & 3, n-tiles 2 (q & 1) + 0/1);
  // the 8 fragment reads of the next phase's set (A: m-tile f / K-slice fk; B: n-tile / K-slice) go
  // out after statements 0-7 (they complete long before the phase's closing lgkmcnt wait), the 4
  // DMA pieces of the phase's half-tile inside statements 9, 11, 13, 15
  auto il_phase = [&](auto m0_c, auto n0_c, const bf16x8_t (&A)[4][2], const bf16x8_t (&B)[4][2], auto rd_b_c,
                      bf16x8_t (&dst)[4][2], const unsigned char* img, int p0, auto kind_c, int t) {
    constexpr int m0 = decltype(m0_c)::value, n0 = decltype(n0_c)::value;
    constexpr bool RDB = decltype(rd_b_c)::value;
    constexpr int kind = decltype(kind_c)::value;
    const unsigned tc = kt0 + (unsigned)(t < KT ? t : KT - 1);
    const unsigned l = lds0 + (t & 1) * BUF + kind * HALF;
    const unsigned so = __builtin_amdgcn_readfirstlane(tc * (kind <= A_HI ? a_kstep : b_kstep));
    const i32x4_t rr = kind <= A_HI ? ra : kind == B_H1 ? rb_hi : rb;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int ks = q >> 3, i = (q >> 1) & 3, j = (q & 1) * 2;
      if (q >= 8 && (q & 1)) {
        const int pc = (q - 9) >> 1;
        g4w_pair_dma(acc[m0 + i][n0 + j], acc[m0 + i][n0 + j + 1], A[i][ks], B[j][ks], B[j + 1][ks],
                     vo[kind][pc], rr, so, l + pc * 4096);
      } else {
        g4w_pair(acc[m0 + i][n0 + j], acc[m0 + i][n0 + j + 1], A[i][ks], B[j][ks], B[j + 1][ks]);
      }
      if (q < 8) {
        const int f = q >> 1, fk = q & 1;
        if constexpr (RDB) dst[f][fk] = frag<BT>(img, p0 + 16 * f, fk, lane);
        else dst[f][fk] = frag<AT>(img, p0 + 16 * f, fk, lane);
      }
    }
  };

  // prologue: K-tiles 0 and 1 in flight; retire A_lo(0) / B(0), read a_lo / b03 of K-tile 0
  issue(K_<A_LO>{}, 0);
  issue(K_<B_H0>{}, 0);
  issue(K_<B_H1>{}, 0);
  issue(K_<A_HI>{}, 0);
  if constexpr (SIDE > 0) {  // W(-2) / L(-2): out-of-range dummies at their stream position
    side_store(K_<0>{});
    side_load(K_<0>{}, std::true_type{});
  }
  issue(K_<A_LO>{}, 1);
  issue(K_<B_H0>{}, 1);
  issue(K_<B_H1>{}, 1);
  issue(K_<A_HI>{}, 1);
  if constexpr (SIDE > 0) {  // W(-1) / L(-1)
    side_store(K_<1>{});
    side_load(K_<1>{}, std::true_type{});
  }
  wait_vm<20 + 2 * S_OPS>();
  bar();
  rdA(a_lo, smem + A_LO * HALF);
  rdB(b03[0], smem + bo03, p03);
  sync(K_<-1>{});  // WAR: P0 restages A_lo of this buffer

  auto ktile_il = [&](int t, auto par_c) {
    constexpr int P = decltype(par_c)::value;
    const unsigned char* buf = smem + P * BUF;
    const unsigned char* nbuf = smem + (P ^ 1) * BUF;
    il_phase(K_<0>{}, K_<0>{}, a_lo, b03[P], std::true_type{}, b47, buf + bo47, p47, K_<A_LO>{}, t + 2);
    sync(K_<20 + 2 * S_OPS>{});
    il_phase(K_<0>{}, K_<4>{}, a_lo, b47, std::false_type{}, a_hi, buf + A_HI * HALF, ap, K_<B_H0>{}, t + 2);
    sync(K_<20 + S_OPS>{});
    il_phase(K_<4>{}, K_<4>{}, a_hi, b47, std::false_type{}, a_lo, nbuf + A_LO * HALF, ap, K_<B_H1>{}, t + 2);
    sync(K_<16 + S_OPS>{});
    il_phase(K_<4>{}, K_<0>{}, a_hi, b03[P], std::true_type{}, b03[P ^ 1], nbuf + bo03, p03, K_<A_HI>{}, t + 2);
    if constexpr (SIDE > 0) {
      side_store(K_<P>{});                   // W(t-2)
      side_load(K_<P>{}, std::false_type{});  // L(t)
    }
    sync(K_<-1>{});
  };
  for (int t = 0; t < KT; t += 2) {
    ktile_il(t, K_<0>{});
    ktile_il(t + 1, K_<1>{});
  }
  wait_vm<0>();  // the clamped tail items are still landing
  if constexpr (SIDE > 0) {  // W(KT-2), W(KT-1)
    side_store(K_<0>{});
    side_store(K_<1>{});
  }
  // the last phase's MFMA results -> the epilogue's accumulator reads: 16 wait states (every
  // other accumulator was last written >= 32 MFMAs earlier)
  g4w_fence(acc);
  if (args.probe & 4) return;
  g4w_epilogue<EPI>(args, acc, tm, tn, wr, wc, lane, sp, u);
}



// ---- persistent 4-wave kernel (config variant 3) ------------------------------------------------
// At K = 4096 the one-shot kernels run ~8 % below hipBLASLt, at K >= 12288 2-3 % (profiles/
// gemm4w_r4_b.txt): a fixed per-tile cost -- the pipeline fill (two K-tiles of DMA waited for with
// nothing to overlap) and the store epilogue.  Here one workgroup per CU walks the work items
// g = blockIdx.x, + gridDim.x, ... and the half-tile DMA stream does not stop at an item boundary:
// the stream slots past the last K-tile of item i (the one-shot kernel's clamped re-loads) fetch
// K-tiles 0 and 1 of item i+1 into the same buffers, in the prologue's order, and the last K-tile's
// phases P2 / P3 already read item i+1's a_lo / b03 fragments.  Item i+1's loop therefore starts
// with its operands in registers, and item i's epilogue stores run while item i+1's first K-tiles
// land.  vmcnt counts the stores too, but they complete out of order with the LDS-DMA loads, so a
// wait may count only younger LOADS: the next item's first waits therefore also wait for the
// epilogue's stores (16-byte stores halve them).  The last two K-tiles are peeled: only there do
// the DMA sources belong to the next item, so its fields are decoded there and the current item's
// buffer descriptors are dead.  The earlier, unpeeled form held both descriptor sets through the
// loop (SGPRs spilled to VGPR lanes) and gave intermittent wrong rows; the peeled form fixed that
// empirically (every test since), but the root cause is NOT pinned down: the suspected VALU write
// of an SGPR (v_readlane reload) ahead of an inline-asm buffer_load was not confirmed --
// tools/sgpr_hazard_check.py found only SALU writers ahead of those loads.  K >= 256.
// Phase schedule: the one-shot 4-wave kernel's.
// STAMP (diagnostic build only: compile with -DLLMCTL_STAMP, then knob gemm_stamp_ptr=<device u32
// buffer>): lane 0 of every wave records s_memtime (low 32 bits) at the start of every phase of its
// first 4 items into LDS and copies them out after each item's epilogue: [block < 32][wave][item <
// 4][STAMPS] (tools/gemm_stamps.py).  The production library carries no diagnostic code.
// Measured-neutral variants tried on this kernel (round 5, profiles/gemm_r5_ab.txt): DMA waits 4 / 8
// pieces tighter (fewer loads in flight), and a phase's DMA pieces spread over the whole phase (wrong
// results: an LDS-DMA interleaved with the phase's fragment reads).
constexpr int STAMPS = 272;
// EXP (diagnostic build, -DLLMCTL_STAMP_EXP=n; results garbage): 1 = no DMA pieces in the loop, 2 = no
// workgroup barriers (waits kept), 3 = no fragment reads -- each phase's cycles without that component.
#ifdef LLMCTL_STAMP
constexpr int STAMP = 1;
#ifdef LLMCTL_STAMP_EXP
constexpr int EXP = LLMCTL_STAMP_EXP;
#else
constexpr int EXP = 0;
#endif
#else
constexpr int STAMP = 0, EXP = 0;
#endif
template <bool AT, bool BT, int EPI, int GROUP, bool RS = false>
__global__ __launch_bounds__(NT4, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm4wp_kernel(G64Args args,
                                                                                                  int n_items) {
  // RS: two 1 KB slots (item parity) of the tile rows' rs values behind the operand buffers
  constexpr int RSB = RS ? 2048 : 0;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * BUF + RSB + (STAMP ? 4 * STAMPS * 4 : 0)];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // lane-constant addressing (DMA voffsets, fragment LDS offsets) is recomputed per item from a
  // laundered thread id: hoisted to kernel entry it stays live across the epilogue, is spilled,
  // and the reloads' compiler vmcnt(0) would wait for the next item's in-flight DMA
  int lane = tid & 63;
  const int wr = wave >> 1, wc = wave & 1;
  constexpr bool PAIRED_B = EPI == EPI_UP_SWIGLU || EPI == EPI_SWIGLU_FWD;
  const long lda = args.lda, ldb = args.ldb;
  const unsigned a_kstep = AT ? (unsigned)(TK * lda * 2) : (unsigned)(TK * 2);
  const unsigned b_kstep = BT ? (unsigned)(TK * ldb * 2) : (unsigned)(TK * 2);

  // work-item fields as plain scalars (a struct of them ended up on the stack)
  auto decode = [&](int bid, int& tm, int& tn, int& sp, int& u, int& KT, unsigned& kt0, i32x4_t& ra, i32x4_t& rb,
                    i32x4_t& rb_hi) __attribute__((always_inline)) {
    int wg;
    sp = -1;
    u = 0;
    if (bid < args.n_main) {
      const int nwg = args.n_main;
      const int q = nwg / 8, rem = nwg % 8, x = bid % 8;
      wg = (x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q) + bid / 8;
    } else {
      const int i = bid - args.n_main;
      u = i / args.splits;
      sp = i - u * args.splits;
      wg = args.n_main + u;
    }
    const int per_group = GROUP * args.tiles_n;
    const int grp = wg / per_group;
    const int gsz = min(GROUP, args.tiles_m - grp * GROUP);
    const int inner = wg - grp * per_group;
    tm = grp * GROUP + inner % gsz;
    tn = inner / gsz;
    KT = sp < 0 ? args.K / TK : args.kt_part;
    kt0 = sp < 0 ? 0u : (unsigned)(sp * args.kt_part);
    const unsigned short* Ab = AT ? args.a + (long)tm * TM : args.a + (long)tm * TM * lda;
    const unsigned short* Bb = PAIRED_B ? args.b + (long)tn * (TN / 2) * ldb
                               : BT ? args.b + (long)tn * TN : args.b + (long)tn * TN * ldb;
    ra = make_rsrc(Ab);
    rb = make_rsrc(Bb);
    rb_hi = PAIRED_B ? make_rsrc(args.b + ((long)args.N + (long)tn * (TN / 2) - TN / 2) * ldb) : rb;
  };

  unsigned vo[4][4];
  auto lane_consts = [&]() __attribute__((always_inline)) {
    int t = tid;
    asm volatile("" : "+v"(t));
    lane = t & 63;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      vo[A_LO][i] = stage_voff<AT, A_LO, NT4>(i, t, lda);
      vo[A_HI][i] = stage_voff<AT, A_HI, NT4>(i, t, lda);
      vo[B_H0][i] = stage_voff<BT, B_H0, NT4>(i, t, ldb);
      vo[B_H1][i] = stage_voff<BT, B_H1, NT4>(i, t, ldb);
    }
  };
  lane_consts();
  const unsigned lds0 = lds_addr(smem) + wave * 1024;
  const int ap = wr * 64;
  const int bo03 = PAIRED_B ? B_H0 * HALF : (B_H0 + wc) * HALF, p03 = PAIRED_B ? wc * 64 : 0;
  const int bo47 = PAIRED_B ? B_H1 * HALF : (B_H0 + wc) * HALF, p47 = PAIRED_B ? wc * 64 : 64;

  int g = blockIdx.x;
  int c_tm, c_tn, c_sp, c_u, c_KT, n_tm, n_tn, n_sp, n_u, n_KT;
  unsigned c_kt0, n_kt0;
  i32x4_t c_ra, c_rb, c_rbh, n_ra, n_rb, n_rbh;
  decode(g, c_tm, c_tn, c_sp, c_u, c_KT, c_kt0, c_ra, c_rb, c_rbh);
  // DMA source of stream slot t: the current item's K-tile t, or (NEXT: an item's last two K-tiles)
  // K-tile t - KT of the next item -- the current item's again after the last item (loads nobody
  // reads, drained before its epilogue)
  auto src = [&](auto next_c, int kind, int t, unsigned& so, i32x4_t& r) __attribute__((always_inline)) {
    constexpr bool NEXT = decltype(next_c)::value;
    const unsigned tc = NEXT ? n_kt0 + (unsigned)(t - c_KT) : c_kt0 + (unsigned)t;
    so = tc * (kind <= A_HI ? a_kstep : b_kstep);
    if (kind <= A_HI) r = NEXT ? n_ra : c_ra;
    else if (kind == B_H1) r = NEXT ? n_rbh : c_rbh;
    else r = NEXT ? n_rb : c_rb;
  };
  auto issue = [&](auto kind_c, int t) __attribute__((always_inline)) {
    constexpr int kind = decltype(kind_c)::value;
    unsigned so;
    i32x4_t r;
    src(std::false_type{}, kind, t, so, r);
    const unsigned l = lds0 + (t & 1) * BUF + kind * HALF;
#pragma unroll
    for (int i = 0; i < 4; ++i) bdma16(r, vo[kind][i], so, l + i * 4096);
  };

  f32x4_t acc[8][8];
  bf16x8_t a_lo[4][2], a_hi[4][2], b47[4][2], b03[2][4][2];
  int sidx = 0;
  auto stamp = [&]() __attribute__((always_inline)) {
    if constexpr (STAMP) {
      const unsigned tt = (unsigned)__builtin_amdgcn_s_memtime();
      if ((tid & 63) == 0 && sidx < STAMPS)
        *reinterpret_cast<unsigned*>(smem + 2 * BUF + RSB + (wave * STAMPS + sidx) * 4) = tt;
      ++sidx;
    }
  };
  auto sync = [&](auto n_c) __attribute__((always_inline)) {
    constexpr int N = decltype(n_c)::value;
    if constexpr (N >= 0) wait_vm<N>();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    if constexpr (EXP != 2) bar();
    stamp();
  };
  auto il_phase = [&](auto m0_c, auto n0_c, const bf16x8_t (&A)[4][2], const bf16x8_t (&B)[4][2], auto rd_b_c,
                      bf16x8_t (&dst)[4][2], const unsigned char* img, int p0, auto kind_c, int t, auto zero_c,
                      auto next_c) __attribute__((always_inline)) {
    constexpr int m0 = decltype(m0_c)::value, n0 = decltype(n0_c)::value;
    constexpr bool ZERO = decltype(zero_c)::value;
    constexpr bool RDB = decltype(rd_b_c)::value;
    constexpr int kind = decltype(kind_c)::value;
    unsigned so;
    i32x4_t rr;
    src(next_c, kind, t, so, rr);
    const unsigned l = lds0 + (t & 1) * BUF + kind * HALF;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int ks = q >> 3, i = (q >> 1) & 3, j = (q & 1) * 2;
      if (EXP != 1 && q >= 8 && (q & 1)) {
        const int pc = (q - 9) >> 1;
        g4w_pair_dma(acc[m0 + i][n0 + j], acc[m0 + i][n0 + j + 1], A[i][ks], B[j][ks], B[j + 1][ks], vo[kind][pc],
                     rr, so, l + pc * 4096);
      } else if (ZERO && q < 8) {
        g4w_pair_z(acc[m0 + i][n0 + j], acc[m0 + i][n0 + j + 1], A[i][ks], B[j][ks], B[j + 1][ks]);
      } else {
        g4w_pair(acc[m0 + i][n0 + j], acc[m0 + i][n0 + j + 1], A[i][ks], B[j][ks], B[j + 1][ks]);
      }
      if (EXP != 3 && q < 8) {
        const int f = q >> 1, fk = q & 1;
        if constexpr (RDB) dst[f][fk] = frag<BT>(img, p0 + 16 * f, fk, lane);
        else dst[f][fk] = frag<AT>(img, p0 + 16 * f, fk, lane);
      }
    }
  };
  auto ktile = [&](int t, auto par_c, auto zero_c, auto next_c) __attribute__((always_inline)) {
    constexpr int P = decltype(par_c)::value;
    const unsigned char* buf = smem + P * BUF;
    const unsigned char* nbuf = smem + (P ^ 1) * BUF;
    il_phase(K_<0>{}, K_<0>{}, a_lo, b03[P], std::true_type{}, b47, buf + bo47, p47, K_<A_LO>{}, t + 2, zero_c, next_c);
    sync(K_<20>{});
    il_phase(K_<0>{}, K_<4>{}, a_lo, b47, std::false_type{}, a_hi, buf + A_HI * HALF, ap, K_<B_H0>{}, t + 2, zero_c,
             next_c);
    sync(K_<20>{});
    il_phase(K_<4>{}, K_<4>{}, a_hi, b47, std::false_type{}, a_lo, nbuf + A_LO * HALF, ap, K_<B_H1>{}, t + 2, zero_c,
             next_c);
    sync(K_<16>{});
    il_phase(K_<4>{}, K_<0>{}, a_hi, b03[P], std::true_type{}, b03[P ^ 1], nbuf + bo03, p03, K_<A_HI>{}, t + 2,
             zero_c, next_c);
    sync(K_<-1>{});
  };

  // K-step 0 fragments of an item's K-tile 0 (buffer 0): a_lo / b03[0]; then lgkmcnt(0) + barrier
  // (WAR: the first phase restages this buffer's A_lo)
  auto first_frags = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) a_lo[i][ks] = frag<AT>(smem + A_LO * HALF, ap + 16 * i, ks, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) b03[0][j][ks] = frag<BT>(smem + bo03, p03 + 16 * j, ks, lane);
    sync(K_<-1>{});
  };
  // RS: wave 0 stages the item's 256 rs values into LDS slot (item parity) with one LDS-DMA piece,
  // issued where no load is outstanding (kernel entry / behind the item-boundary drain): it is then
  // the OLDEST load, retired by the first counted wait that also retires younger pieces (loads
  // retire in order), so every count in the loop still holds; the K-loop's barriers publish it to
  // the other waves long before the epilogue.  A slot is rewritten two items later, after the
  // barriers of the item in between (no wave still reads it).
  int it = 0;
  auto rs_issue = [&]() __attribute__((always_inline)) {
    if constexpr (RS) {
      if (wave == 0)
        bdma16(make_rsrc(args.rs + (long)c_tm * TM), (unsigned)(tid & 63) * 16u, 0u,
               lds_addr(smem) + 2 * BUF + (it & 1) * 1024);
    }
  };
  rs_issue();
  // prologue (first item only): K-tiles 0 and 1 in flight; retire A_lo(0) / B(0)
  issue(K_<A_LO>{}, 0);
  issue(K_<B_H0>{}, 0);
  issue(K_<B_H1>{}, 0);
  issue(K_<A_HI>{}, 0);
  issue(K_<A_LO>{}, 1);
  issue(K_<B_H0>{}, 1);
  issue(K_<B_H1>{}, 1);
  issue(K_<A_HI>{}, 1);
  wait_vm<20>();
  bar();

  while (true) {
    lane_consts();
    // the item's K-tile 0 is in buffer 0 (the prologue's, or the previous item's stream tail behind
    // its last waits and barrier): its first fragments are read here, so no fragment is carried
    // through the loop's back-edge (nor live across the epilogue)
    first_frags();
    // K-tile 0 starts every accumulator from C = 0 (KT >= 4, even)
    ktile(0, K_<0>{}, std::true_type{}, std::false_type{});
    ktile(1, K_<1>{}, std::false_type{}, std::false_type{});
    for (int t = 2; t < c_KT - 2; t += 2) {
      ktile(t, K_<0>{}, std::false_type{}, std::false_type{});
      ktile(t + 1, K_<1>{}, std::false_type{}, std::false_type{});
    }
    const bool has_next = g + (int)gridDim.x < n_items;
    decode(has_next ? g + (int)gridDim.x : g, n_tm, n_tn, n_sp, n_u, n_KT, n_kt0, n_ra, n_rb, n_rbh);
    ktile(c_KT - 2, K_<0>{}, std::false_type{}, std::true_type{});
    ktile(c_KT - 1, K_<1>{}, std::false_type{}, std::true_type{});
    g4w_fence(acc);
    if (!has_next) wait_vm<0>();  // the re-loads of the last item's K-tiles 0 / 1 are still landing
    stamp();
    g4w_epilogue<EPI, RS>(args, acc, c_tm, c_tn, wr, wc, lane, c_sp, c_u,
                          reinterpret_cast<const float*>(smem + 2 * BUF + (it & 1) * 1024));
    if constexpr (STAMP) {
      wait_vm<0>();
      stamp();
      __builtin_amdgcn_s_waitcnt(0xC07F);
      const int it = (g - (int)blockIdx.x) / (int)gridDim.x;
      unsigned* out = reinterpret_cast<unsigned*>(args.stamp_ptr);
      if (out != nullptr && blockIdx.x < 32 && it < 4)
        for (int e = (tid & 63); e < STAMPS; e += 64)
          out[((blockIdx.x * 4 + wave) * 4 + it) * STAMPS + e] =
              *reinterpret_cast<const unsigned*>(smem + 2 * BUF + RSB + (wave * STAMPS + e) * 4);
      wait_vm<0>();
      sidx = 0;
    }
    if (!has_next) break;
    // vmcnt accounting at an item boundary: the stream slots of the last two K-tiles already hold
    // the next item's K-tiles 0 / 1 (16 DMA pieces), and the epilogue adds its 32 stores behind
    // them.  vmcnt counts loads and stores together but they RETIRE out of order, so a counted
    // wait (the next item's first wait_vm<20>, which assumes only DMA pieces are younger) could
    // pass while the K-tile 0 pieces have not landed.  Draining here makes every later count
    // exact again: the first fragment reads of the next item then see landed data (this wait
    // costs one DMA latency per item, ~0.3 % at K = 4096).  Unconditional: the undrained form
    // gave intermittent wrong rows.
    wait_vm<0>();
    g += (int)gridDim.x;
    c_tm = n_tm, c_tn = n_tn, c_sp = n_sp, c_u = n_u, c_KT = n_KT, c_kt0 = n_kt0;
    c_ra = n_ra, c_rb = n_rb, c_rbh = n_rbh;
    ++it;
    rs_issue();
  }
}

// sum of the split partials of tail tile u (grouped-order position n_main + u) + epilogue;
// thread = 8 consecutive columns of one row
template <int EPI, int GROUP, bool RS = false>
__global__ __launch_bounds__(256) void gemm64_split_reduce(G64Args args) {
  const int u = blockIdx.x / (TM * TN / 8 / 256);
  const int e = (blockIdx.x % (TM * TN / 8 / 256)) * 256 + threadIdx.x;  // 8-column chunk in the tile
  const int row = e / (TN / 8), col = (e % (TN / 8)) * 8;
  const int wg = args.n_main + u;
  const int per_group = GROUP * args.tiles_n;
  const int grp = wg / per_group;
  const int gsz = min(GROUP, args.tiles_m - grp * GROUP);
  const int inner = wg - grp * per_group;
  const int tm = grp * GROUP + inner % gsz, tn = inner / gsz;
  float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const float* W = args.ws + (long)u * args.splits * (TM * TN) + row * TN + col;
  for (int sp = 0; sp < args.splits; ++sp) {
    const f32x4_t x0 = *reinterpret_cast<const f32x4_t*>(W + (long)sp * (TM * TN));
    const f32x4_t x1 = *reinterpret_cast<const f32x4_t*>(W + (long)sp * (TM * TN) + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] += x0[j];
      v[4 + j] += x1[j];
    }
  }
  if constexpr (RS) {
    const float r = args.rs[(long)tm * TM + row];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] *= r;
  }
  if constexpr (EPI == EPI_SWIGLU_FWD) {
    // the paired tile's gate cols [0, 128) and their up partners 128 + [0, 128): a thread of the gate
    // half sums its partners too and writes act = silu(g) * u (as the main epilogue, on bf16 g / u)
    if (col >= TN / 2) return;
    float w2[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int sp = 0; sp < args.splits; ++sp) {
      const f32x4_t x0 = *reinterpret_cast<const f32x4_t*>(W + TN / 2 + (long)sp * (TM * TN));
      const f32x4_t x1 = *reinterpret_cast<const f32x4_t*>(W + TN / 2 + (long)sp * (TM * TN) + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        w2[j] += x0[j];
        w2[4 + j] += x1[j];
      }
    }
    if constexpr (RS) {
      const float r = args.rs[(long)tm * TM + row];
#pragma unroll
      for (int j = 0; j < 8; ++j) w2[j] *= r;
    }
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gg = bf2f(f2bf(v[j])), uu = bf2f(f2bf(w2[j]));
      o[j] = gg * (1.f / (1.f + __expf(-gg))) * uu;
    }
    store8(args.c + ((long)tm * TM + row) * args.ldc + (long)tn * (TN / 2) + col, o);
    return;
  }
  if constexpr (EPI == EPI_ROPE_QKV) {
    // the main epilogue's RoPE / head split: a thread of the first half of a head (d < 64) also sums
    // its rotation partners d + 64 and writes both halves
    const int hh = col >> 7, d = col & 127;
    if (d >= 64) return;
    float w2[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int sp = 0; sp < args.splits; ++sp) {
      const f32x4_t x0 = *reinterpret_cast<const f32x4_t*>(W + 64 + (long)sp * (TM * TN));
      const f32x4_t x1 = *reinterpret_cast<const f32x4_t*>(W + 64 + (long)sp * (TM * TN) + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        w2[j] += x0[j];
        w2[4 + j] += x1[j];
      }
    }
    const int h = 2 * tn + hh, nrot = args.nq + args.nkv;
    unsigned short* dst0;
    long dst_ld;
    if (h < args.nq) {
      dst0 = args.c + (long)h * 128;
      dst_ld = (long)args.nq * 128;
    } else if (h < nrot) {
      dst0 = args.out2 + (long)(h - args.nq) * 128;
      dst_ld = (long)args.nkv * 128;
    } else {
      dst0 = args.out3 + (long)(h - nrot) * 128;
      dst_ld = (long)args.nkv * 128;
    }
    const long t = (long)tm * TM + row;
    float o1[8], o2[8];
    if (h < nrot) {  // as rope_fwd_kernel on the bf16-stored projection
      const long p = args.pos ? (long)args.pos[t] : (long)(t % args.seq);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float a = bf2f(f2bf(v[j])), b = bf2f(f2bf(w2[j]));
        const float cs = args.cosT[p * 64 + d + j], sn = args.sinT[p * 64 + d + j];
        o1[j] = a * cs - b * sn;
        o2[j] = b * cs + a * sn;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        o1[j] = v[j];
        o2[j] = w2[j];
      }
    }
    store8(dst0 + t * dst_ld + d, o1);
    store8(dst0 + t * dst_ld + 64 + d, o2);
    return;
  }
  if constexpr (epi_f32(EPI)) {
    f32x4_t* pf = reinterpret_cast<f32x4_t*>(reinterpret_cast<float*>(args.c) + (long)(tm * TM + row) * args.ldc + tn * TN + col);
    f32x4_t lo = {v[0], v[1], v[2], v[3]}, hi = {v[4], v[5], v[6], v[7]};
    if constexpr (EPI == EPI_ACC_F32) {
      lo += pf[0];
      hi += pf[1];
    }
    pf[0] = lo;
    pf[1] = hi;
    return;
  }
  unsigned short* p = args.c + (long)(tm * TM + row) * args.ldc + tn * TN + col;
  if constexpr (EPI == EPI_SWIGLU_BWD) {
    const unsigned short* gp = args.aux + (p - args.c);
    float gf[8], uf[8], dg[8], du[8];
    load8(gp, gf);
    load8(gp + args.N, uf);
#pragma unroll
    for (int j = 0; j < 8; ++j) swiglu_bwd1(v[j], gf[j], uf[j], dg[j], du[j]);
    store8(p, dg);
    store8(p + args.N, du);
    return;
  }
  if constexpr (EPI == EPI_ACC) {
    float old[8];
    load8(p, old);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += old[j];
  }
  store8(p, v);
}

// schedule variant (config / 100 % 10): 3 = the persistent 4-wave kernel, >= 4 = the one-shot 4-wave
// kernel, 0-2 = the 8-wave kernel (the SwiGLU-backward epilogue: always the 8-wave kernel).  Retired
// (measured slower, aliased here): the 8-wave schedules 0 / 2 / 3 and persistent 8-wave kernel (5;
// profiles/gemm_persistent_r3.txt), the 4-wave K-step-major kernel (4) and the 4-wave phase
// orderings 6-8 (profiles/ab_gemm64_config_r4.log), register-staged B (profiles/gemm_regstage_ab_r4.txt)
template <bool AT, bool BT, int EPI, int GROUP, bool RS = false>
void launch_g(const G64Args& g, int variant) {
  const int n_items = g.n_main + (g.tiles_m * g.tiles_n - g.n_main) * g.splits;
  const dim3 grid(n_items);
  bool launched = false;
  if constexpr (RS) {  // row-scaled epilogue: the persistent kernel only
    LLMCTL_CHECK(variant == 3 && g.K >= 4 * TK, "gemm64 row-scaled epilogue: persistent schedule (variant 3), K >= 256");
    hipLaunchKernelGGL((gemm4wp_kernel<AT, BT, EPI, GROUP, true>), dim3(min(n_items, num_cus())), dim3(NT4), 0, stream(),
                       g, n_items);
    launched = true;
  } else if constexpr (EPI != EPI_SWIGLU_BWD) {
    if (variant == 3 && g.K >= 4 * TK) {  // the persistent kernel peels two K-tiles per item
      hipLaunchKernelGGL((gemm4wp_kernel<AT, BT, EPI, GROUP>), dim3(min(n_items, num_cus())), dim3(NT4), 0, stream(), g,
                         n_items);
      launched = true;
    } else if (variant >= 3) {
      hipLaunchKernelGGL((gemm4w_kernel<AT, BT, EPI, GROUP>), grid, dim3(NT4), 0, stream(), g);
      launched = true;
    }
  }
  if constexpr (!RS)
    if (!launched) hipLaunchKernelGGL((gemm64_kernel<AT, BT, EPI, GROUP>), grid, dim3(NTHR), 0, stream(), g);
  const int n_tail = g.tiles_m * g.tiles_n - g.n_main;
  if (n_tail > 0)
    hipLaunchKernelGGL((gemm64_split_reduce<EPI, GROUP, RS>), dim3(n_tail * (TM * TN / 8 / 256)), dim3(256), 0,
                       stream(), g);
}

// config = group (tile-rows per tile-order group: 4 / 8) + 100 * schedule variant
//          + 1000 * split (0: automatic tail split, 1: none, S >= 2: S K-ranges when legal)
template <bool AT, bool BT, int EPI, bool RS = false>
void launch(const G64Args& g, int config) {
  const int group = config % 100, variant = (config / 100) % 10;
  if (group == 8) launch_g<AT, BT, EPI, 8, RS>(g, variant);
  else launch_g<AT, BT, EPI, 4, RS>(g, variant);
}

// Tail split plan: tiles of the last, partial round (when it is at most half full) are cut into
// S K-ranges (KT % S == 0, an even number >= 4 of K-tiles each).  Estimated cost in tile-times:
//   ceil(n_tail * S / CUs) / S   + workspace traffic (write + re-read of S fp32 partial tiles,
//   ~0.5 us per partial tile at ~4 TB/s) in units of one tile's run time.
void plan_split(G64Args& g, int mode) {
  const int tiles = g.tiles_m * g.tiles_n, KT = g.K / TK, cus = num_cus();
  g.n_main = tiles;
  g.splits = 1;
  g.kt_part = KT;
  g.ws = nullptr;
  if (mode == 1) return;
  // tiles of the last round; a forced split of a whole number of rounds splits the last round
  const int n_tail = tiles % cus ? tiles % cus : (mode >= 2 ? min(tiles, cus) : 0);
  // auto: only a last round at most half full (measured: a 69 %-full round of the GPT-7B
  // down-projection wgrad lost 2 % to the workspace traffic; 37 % / 12 % / 50 % ones gained
  // 8.6 % / 3.6 % / 18 %, profiles/gemm64_split_r2.txt)
  if (n_tail == 0 || (mode == 0 && n_tail * 2 > cus)) return;
  // one tile's time on one CU at ~1.4 PF chip-wide
  const double tile_us = 2.0 * TM * TN * (double)g.K / (1.4e15 / cus) * 1e6;
  double best = 1.0;  // unsplit tail: one full tile-time
  int best_s = 1;
  const int cands[] = {2, 3, 4, 6, 8, 12, 16};
  for (int S : cands) {
    if (mode >= 2 && S != mode) continue;
    if (KT % S || (KT / S) % 2 || KT / S < 4) continue;
    const double rounds = (double)((n_tail * S + cus - 1) / cus) / S;
    const double traffic = 2.0 * n_tail * S * (TM * TN * 4.0) / 4e12 * 1e6 / tile_us;
    const double cost = rounds + traffic + 0.1;  // + reduction launch / pipeline ramp of the items
    if (cost < best || mode >= 2) {
      best = cost;
      best_s = S;
    }
  }
  if (best_s == 1) return;
  g.n_main = tiles - n_tail;
  g.splits = best_s;
  g.kt_part = KT / best_s;
}

}  // namespace

bool gemm64_supported(long M, long N, long K) { return M % TM == 0 && N % TN == 0 && K % (2 * TK) == 0 && K > 0; }

// out[M,N] (+)= A·B^T, operand storage by at / bt; M, N multiples of 256, K of 128.
void gemm64_ex(const at::Tensor& a, const at::Tensor& b, at::Tensor& out, bool at_, bool bt_, bool accumulate,
               int64_t config) {
  LLMCTL_CHECK(a.dim() == 2 && b.dim() == 2 && out.dim() == 2, "gemm64_ex: 2-D operands");
  const bool f32_out = out.scalar_type() == at::kFloat;
  LLMCTL_CHECK(a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16 &&
                   (out.scalar_type() == at::kBFloat16 || (f32_out && at_ && bt_)),
               "gemm64_ex: bf16 operands, bf16 output (fp32 output: wgrad layout only)");
  LLMCTL_CHECK(a.is_cuda() && b.is_cuda() && out.is_cuda(), "gemm64_ex: GPU tensors");
  LLMCTL_CHECK(a.stride(1) == 1 && b.stride(1) == 1 && out.stride(1) == 1, "gemm64_ex: unit inner stride");
  const long M = at_ ? a.size(1) : a.size(0);
  const long K = at_ ? a.size(0) : a.size(1);
  const long N = bt_ ? b.size(1) : b.size(0);
  const long Kb = bt_ ? b.size(0) : b.size(1);
  LLMCTL_CHECK(K == Kb, "gemm64_ex: K mismatch (", K, " vs ", Kb, ")");
  LLMCTL_CHECK(out.size(0) == M && out.size(1) == N, "gemm64_ex: out must be [M,N]");
  LLMCTL_CHECK(gemm64_supported(M, N, K), "gemm64_ex: M,N multiples of 256, K of 128 (got ", M, "x", N, "x", K, ")");
  LLMCTL_CHECK(a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0 && out.stride(0) % 4 == 0 &&
                   (reinterpret_cast<uintptr_t>(a.data_ptr()) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(b.data_ptr()) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(out.data_ptr()) & (f32_out ? 15 : 7)) == 0,
               "gemm64_ex: 16-byte aligned operand rows");
  // 32-bit buffer offsets: the farthest byte any tile's DMA addresses from its tile origin
  const long a_span = at_ ? K * a.stride(0) * 2 : (long)TM * a.stride(0) * 2;
  const long b_span = bt_ ? K * b.stride(0) * 2 : (long)TN * b.stride(0) * 2;
  LLMCTL_CHECK(a_span < (1L << 31) && b_span < (1L << 31), "gemm64_ex: operand too large for 32-bit offsets");
  const c10::DeviceGuard dg(a.device());
  G64Args g{reinterpret_cast<const unsigned short*>(a.data_ptr()), reinterpret_cast<const unsigned short*>(b.data_ptr()),
            reinterpret_cast<unsigned short*>(out.data_ptr()), a.stride(0), b.stride(0), out.stride(0),
            (int)M, (int)N, (int)K, (int)(M / TM), (int)(N / TN), 0, 1, 0, nullptr, nullptr};
  g.probe = (int)knob("gemm_probe", 0);
  g.stamp_ptr = (unsigned long)knob("gemm_stamp_ptr", 0);
  plan_split(g, (int)(config / 1000));
  at::Tensor ws;
  if (g.splits > 1) {
    ws = at::empty({(long)(g.tiles_m * g.tiles_n - g.n_main) * g.splits * TM * TN}, a.options().dtype(at::kFloat));
    g.ws = ws.data_ptr<float>();
  }
  const int grp = (int)(config % 1000);
  if (f32_out) {  // fp32 main gradients
    if (accumulate) launch<true, true, EPI_ACC_F32>(g, grp);
    else launch<true, true, EPI_STORE_F32>(g, grp);
    return;
  }
  const int sel = (at_ ? 4 : 0) | (bt_ ? 2 : 0) | (accumulate ? 1 : 0);
  switch (sel) {
    case 0: launch<false, false, EPI_STORE>(g, grp); break;
    case 1: launch<false, false, EPI_ACC>(g, grp); break;
    case 2: launch<false, true, EPI_STORE>(g, grp); break;
    case 3: launch<false, true, EPI_ACC>(g, grp); break;
    case 4: launch<true, false, EPI_STORE>(g, grp); break;
    case 5: launch<true, false, EPI_ACC>(g, grp); break;
    case 6: launch<true, true, EPI_STORE>(g, grp); break;
    default: launch<true, true, EPI_ACC>(g, grp); break;
  }
}

// Down-projection data gradient fused with the SwiGLU backward:
//   dAct = dy · W_down  (dy [M, H], W_down [H, F]; gemm64's dgrad layout, W read K-major)
//   dgu[:, :F] = dAct * u * sig(g) * (1 + g (1 - sig(g))),  dgu[:, F:] = dAct * silu(g)
// with g = gu[:, :F], u = gu[:, F:].  Returns dgu [M, 2F].
at::Tensor gemm64_swiglu_dgrad(const at::Tensor& dy, const at::Tensor& w, const at::Tensor& gu, int64_t config) {
  LLMCTL_CHECK(dy.dim() == 2 && w.dim() == 2 && gu.dim() == 2, "gemm64_swiglu_dgrad: 2-D operands");
  LLMCTL_CHECK(dy.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16 && gu.scalar_type() == at::kBFloat16,
               "gemm64_swiglu_dgrad: bf16 operands");
  LLMCTL_CHECK(dy.is_cuda() && w.is_cuda() && gu.is_cuda(), "gemm64_swiglu_dgrad: GPU tensors");
  LLMCTL_CHECK(dy.stride(1) == 1 && w.stride(1) == 1 && gu.is_contiguous(), "gemm64_swiglu_dgrad: row-major operands");
  const long M = dy.size(0), K = dy.size(1), N = w.size(1);
  LLMCTL_CHECK(w.size(0) == K, "gemm64_swiglu_dgrad: dy [M,H] vs W [H,F]");
  LLMCTL_CHECK(gu.size(0) == M && gu.size(1) == 2 * N, "gemm64_swiglu_dgrad: gu must be [M, 2F]");
  LLMCTL_CHECK(gemm64_supported(M, N, K), "gemm64_swiglu_dgrad: M,F multiples of 256, H of 128 (got ", M, "x", N, "x", K,
               ")");
  LLMCTL_CHECK(dy.stride(0) % 8 == 0 && w.stride(0) % 8 == 0 && (reinterpret_cast<uintptr_t>(dy.data_ptr()) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(w.data_ptr()) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(gu.data_ptr()) & 15) == 0,
               "gemm64_swiglu_dgrad: 16-byte aligned operand rows");
  const long a_span = (long)TM * dy.stride(0) * 2, b_span = K * w.stride(0) * 2;
  LLMCTL_CHECK(a_span < (1L << 31) && b_span < (1L << 31), "gemm64_swiglu_dgrad: operand too large for 32-bit offsets");
  const c10::DeviceGuard dg(dy.device());
  auto dgu = at::empty_like(gu);
  G64Args g{reinterpret_cast<const unsigned short*>(dy.data_ptr()), reinterpret_cast<const unsigned short*>(w.data_ptr()),
            reinterpret_cast<unsigned short*>(dgu.data_ptr()), dy.stride(0), w.stride(0), 2 * N,
            (int)M, (int)N, (int)K, (int)(M / TM), (int)(N / TN), 0, 1, 0, nullptr,
            reinterpret_cast<const unsigned short*>(gu.data_ptr())};
  plan_split(g, (int)(config / 1000));
  at::Tensor ws;
  if (g.splits > 1) {
    ws = at::empty({(long)(g.tiles_m * g.tiles_n - g.n_main) * g.splits * TM * TN}, dy.options().dtype(at::kFloat));
    g.ws = ws.data_ptr<float>();
  }
  launch<false, true, EPI_SWIGLU_BWD>(g, (int)(config % 1000));
  return dgu;
}

template <int EPI, int SIDE>
void launch_side(const G64Args& g, int variant) {
  const int n_items = g.n_main + (g.tiles_m * g.tiles_n - g.n_main) * g.splits;
  if (variant >= 3)  // the one-shot 4-wave kernel (launch_g's variant map; no persistent side-job kernel)
    hipLaunchKernelGGL((gemm4w_kernel<true, true, EPI, 4, SIDE>), dim3(n_items), dim3(NT4), 0, stream(), g);
  else
    hipLaunchKernelGGL((gemm64_kernel<true, true, EPI, 4, SIDE>), dim3(n_items), dim3(NTHR), 0, stream(), g);
  const int n_tail = g.tiles_m * g.tiles_n - g.n_main;
  if (n_tail > 0)
    hipLaunchKernelGGL((gemm64_split_reduce<EPI, 4>), dim3(n_tail * (TM * TN / 8 / 256)), dim3(256), 0, stream(), g);
}

template <int EPI>
void launch_side_ch(const G64Args& g, int ch, int variant) {
  if (ch == 1) launch_side<EPI, 1>(g, variant);
  else launch_side<EPI, 2>(g, variant);
}

// chunks of 1024 elements per K-tile the side job needs for E = T * F elements over the K-tiles
// of an [M, N] x K wgrad (0: more than 2, or offsets past 32 bits — not supported)
int side_chunks(long M, long N, long K, long T, long F) {
  const long ktiles = (M / TM) * (N / TN) * (K / TK), E = T * F;
  if (E * 4 >= (1L << 31) || F % 2) return 0;
  for (int ch = 1; ch <= 2; ++ch)
    if (ktiles * 1024 * ch >= E && ktiles * 1024 * ch < (1L << 32) && F >= 1024L * ch) return ch;
  return 0;
}

// Down-projection weight gradient with the SwiGLU backward as a side job (see "side job" above):
//   gw (+)= dy^T act               dy [T, H], act [T, F]  (wgrad layout; gw [H, F] bf16 or fp32)
//   dgu = swiglu_bwd(dact, gu)     dact [T, F], gu [T, 2F] -> returned [T, 2F]
at::Tensor gemm64_wgrad_swiglu(const at::Tensor& dy, const at::Tensor& act, at::Tensor& gw, bool accumulate,
                               const at::Tensor& dact, const at::Tensor& gu, int64_t config) {
  LLMCTL_CHECK(dy.dim() == 2 && act.dim() == 2 && gw.dim() == 2 && dact.dim() == 2 && gu.dim() == 2,
               "gemm64_wgrad_swiglu: 2-D operands");
  const bool f32_out = gw.scalar_type() == at::kFloat;
  LLMCTL_CHECK(dy.scalar_type() == at::kBFloat16 && act.scalar_type() == at::kBFloat16 &&
                   dact.scalar_type() == at::kBFloat16 && gu.scalar_type() == at::kBFloat16 &&
                   (f32_out || gw.scalar_type() == at::kBFloat16),
               "gemm64_wgrad_swiglu: bf16 operands, bf16 / fp32 weight gradient");
  LLMCTL_CHECK(dy.is_cuda() && act.is_cuda() && gw.is_cuda() && dact.is_cuda() && gu.is_cuda(),
               "gemm64_wgrad_swiglu: GPU tensors");
  const long T = dy.size(0), M = dy.size(1), N = act.size(1);
  LLMCTL_CHECK(act.size(0) == T && gw.size(0) == M && gw.size(1) == N, "gemm64_wgrad_swiglu: dy [T,H], act [T,F], gw [H,F]");
  LLMCTL_CHECK(dact.is_contiguous() && gu.is_contiguous() && dact.size(0) == T && dact.size(1) == N &&
                   gu.size(0) == T && gu.size(1) == 2 * N,
               "gemm64_wgrad_swiglu: contiguous dact [T, F], gu [T, 2F]");
  LLMCTL_CHECK(dy.stride(1) == 1 && act.stride(1) == 1 && gw.stride(1) == 1, "gemm64_wgrad_swiglu: unit inner stride");
  LLMCTL_CHECK(gemm64_supported(M, N, T), "gemm64_wgrad_swiglu: H, F multiples of 256, T of 128 (got ", M, "x", N, "x", T,
               ")");
  LLMCTL_CHECK(dy.stride(0) % 8 == 0 && act.stride(0) % 8 == 0 && gw.stride(0) % 4 == 0 &&
                   (reinterpret_cast<uintptr_t>(dy.data_ptr()) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(act.data_ptr()) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(gw.data_ptr()) & (f32_out ? 15 : 7)) == 0 &&
                   (reinterpret_cast<uintptr_t>(dact.data_ptr()) & 3) == 0 &&
                   (reinterpret_cast<uintptr_t>(gu.data_ptr()) & 3) == 0,
               "gemm64_wgrad_swiglu: aligned operand rows");
  LLMCTL_CHECK(T * dy.stride(0) * 2 < (1L << 31) && T * act.stride(0) * 2 < (1L << 31),
               "gemm64_wgrad_swiglu: operand too large for 32-bit offsets");
  const int ch = side_chunks(M, N, T, T, N);
  LLMCTL_CHECK(ch > 0, "gemm64_wgrad_swiglu: side job does not fit (", T, " x ", N, " elements over ", M, " x ", N,
               " x ", T, ")");
  const c10::DeviceGuard dg(dy.device());
  auto dgu = at::empty_like(gu);
  G64Args g{reinterpret_cast<const unsigned short*>(dy.data_ptr()), reinterpret_cast<const unsigned short*>(act.data_ptr()),
            reinterpret_cast<unsigned short*>(gw.data_ptr()), dy.stride(0), act.stride(0), gw.stride(0),
            (int)M, (int)N, (int)T, (int)(M / TM), (int)(N / TN), 0, 1, 0, nullptr, nullptr};
  g.s_dact = reinterpret_cast<const unsigned short*>(dact.data_ptr());
  g.s_gu = reinterpret_cast<const unsigned short*>(gu.data_ptr());
  g.s_dgu = reinterpret_cast<unsigned short*>(dgu.data_ptr());
  g.s_E = (unsigned)(T * N);
  g.s_F = (int)N;
  plan_split(g, (int)(config / 1000));
  at::Tensor ws;
  if (g.splits > 1) {
    ws = at::empty({(long)(g.tiles_m * g.tiles_n - g.n_main) * g.splits * TM * TN}, dy.options().dtype(at::kFloat));
    g.ws = ws.data_ptr<float>();
  }
  const int variant = (int)((config % 1000) / 100);
  if (f32_out) {
    if (accumulate) launch_side_ch<EPI_ACC_F32>(g, ch, variant);
    else launch_side_ch<EPI_STORE_F32>(g, ch, variant);
  } else {
    if (accumulate) launch_side_ch<EPI_ACC>(g, ch, variant);
    else launch_side_ch<EPI_STORE>(g, ch, variant);
  }
  return dgu;
}

// Gate/up projection fused with SwiGLU (serving prefill): act [M, F] = silu(x Wg^T) * (x Wu^T) with
// W_up = [Wg; Wu] [2F, K] (forward layout, both operands K-contiguous); M % 256, F % 128, K % 128.
void check_rstd(const c10::optional<at::Tensor>& rstd, long M, const char* who) {
  if (!rstd.has_value() || !rstd->defined()) return;
  LLMCTL_CHECK(rstd->is_cuda() && rstd->scalar_type() == at::kFloat && rstd->is_contiguous() && rstd->numel() == M, who,
               ": rstd must be a contiguous fp32 GPU tensor [M]");
}

// persistent schedule (variant 3) of a config, keeping its group and split fields
int persistent_config(int64_t config) { return (int)((config / 1000) * 1000 + 300 + config % 100); }

at::Tensor gemm64_swiglu_fwd(const at::Tensor& x, const at::Tensor& w, int64_t config,
                             const c10::optional<at::Tensor>& rstd) {
  LLMCTL_CHECK(x.dim() == 2 && w.dim() == 2 && x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16 &&
                   x.is_cuda() && w.is_cuda() && x.stride(1) == 1 && w.is_contiguous(),
               "gemm64_swiglu_fwd: bf16 GPU x [M, K] (unit inner stride), contiguous W_up [2F, K]");
  const long M = x.size(0), K = x.size(1), F = w.size(0) / 2;
  LLMCTL_CHECK(w.size(1) == K && w.size(0) == 2 * F, "gemm64_swiglu_fwd: W_up must be [2F, K]");
  LLMCTL_CHECK(M % TM == 0 && F % (TN / 2) == 0 && K % (2 * TK) == 0 && K > 0,
               "gemm64_swiglu_fwd: M % 256, F % 128, K % 128 (got ", M, "x", F, "x", K, ")");
  LLMCTL_CHECK(x.stride(0) % 8 == 0 && (reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(w.data_ptr()) & 15) == 0,
               "gemm64_swiglu_fwd: 16-byte aligned operand rows");
  LLMCTL_CHECK((long)TM * x.stride(0) * 2 < (1L << 31) && (long)TN * K * 2 < (1L << 31),
               "gemm64_swiglu_fwd: operand too large for 32-bit offsets");
  const c10::DeviceGuard dg(x.device());
  auto act = at::empty({M, F}, x.options());
  G64Args g{reinterpret_cast<const unsigned short*>(x.data_ptr()), reinterpret_cast<const unsigned short*>(w.data_ptr()),
            reinterpret_cast<unsigned short*>(act.data_ptr()), x.stride(0), K, F,
            (int)M, (int)F, (int)K, (int)(M / TM), (int)(F / (TN / 2)), 0, 1, 0, nullptr, nullptr};
  // tail split (config / 1000, 0 = automatic): split items store the paired tile's fp32 partials and
  // gemm64_split_reduce applies the SwiGLU (e.g. 4,096 tokens of GPT-7B: 1,376 tiles = 5.375 rounds).
  // Native knob swiglu_fwd_split = 0: whole tiles only (A/B)
  plan_split(g, knob("swiglu_fwd_split", 1) ? (int)(config / 1000) : 1);
  at::Tensor ws;
  if (g.splits > 1) {
    ws = at::empty({(long)(g.tiles_m * g.tiles_n - g.n_main) * g.splits * TM * TN}, x.options().dtype(at::kFloat));
    g.ws = ws.data_ptr<float>();
  }
  check_rstd(rstd, M, "gemm64_swiglu_fwd");
  if (rstd.has_value() && rstd->defined()) {
    LLMCTL_CHECK(K >= 4 * TK, "gemm64_swiglu_fwd: row-scaled form needs K >= 256");
    g.rs = rstd->data_ptr<float>();
    launch<false, false, EPI_SWIGLU_FWD, true>(g, persistent_config(config) % 1000);
  } else {
    launch<false, false, EPI_SWIGLU_FWD>(g, (int)(config % 1000));
  }
  return act;
}

// QKV projection with RoPE + head split in the epilogue (training forward): x [T, K] (T % 256),
// w [(nq + 2 nkv) * 128, K], cos / sin [P][64] fp32, pos int32 [T] or empty (t % seq).
std::tuple<at::Tensor, at::Tensor, at::Tensor> gemm64_qkv_rope(const at::Tensor& x, const at::Tensor& w,
                                                               const at::Tensor& cosT, const at::Tensor& sinT,
                                                               const c10::optional<at::Tensor>& pos, int64_t nq,
                                                               int64_t nkv, int64_t seq, int64_t config) {
  LLMCTL_CHECK(x.dim() == 2 && w.dim() == 2 && x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16 &&
                   x.is_cuda() && w.is_cuda() && x.stride(1) == 1 && w.is_contiguous(),
               "gemm64_qkv_rope: bf16 GPU x [T, K] (unit inner stride), contiguous W [(nq+2nkv)*128, K]");
  const long T = x.size(0), K = x.size(1), N = w.size(0);
  LLMCTL_CHECK(w.size(1) == K && N == (nq + 2 * nkv) * 128 && nq % 2 == 0 && nkv % 2 == 0,
               "gemm64_qkv_rope: head_dim 128, even head counts, W [(nq+2nkv)*128, K]");
  LLMCTL_CHECK(T % TM == 0 && K % (2 * TK) == 0 && K > 0, "gemm64_qkv_rope: T % 256, K % 128 (got ", T, "x", K, ")");
  LLMCTL_CHECK(cosT.scalar_type() == at::kFloat && sinT.scalar_type() == at::kFloat && cosT.is_contiguous() &&
                   sinT.is_contiguous() && cosT.dim() == 2 && cosT.size(1) == 64 && sinT.sizes() == cosT.sizes(),
               "gemm64_qkv_rope: fp32 cos/sin tables [P][64]");
  LLMCTL_CHECK(x.stride(0) % 8 == 0 && (reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0 &&
                   (long)TM * x.stride(0) * 2 < (1L << 31) && (long)TN * K * 2 < (1L << 31),
               "gemm64_qkv_rope: 16-byte aligned rows / 32-bit offsets");
  const bool has_pos = pos.has_value() && pos->defined() && pos->numel() > 0;
  if (has_pos) {
    LLMCTL_CHECK(pos->scalar_type() == at::kInt && pos->is_contiguous() && pos->numel() == T,
                 "gemm64_qkv_rope: int32 positions [T]");
  } else {
    LLMCTL_CHECK(cosT.size(0) >= seq, "gemm64_qkv_rope: tables shorter than seq");
  }
  const c10::DeviceGuard dg(x.device());
  auto q = at::empty({T, nq, 128}, x.options());
  auto k = at::empty({T, nkv, 128}, x.options());
  auto v = at::empty({T, nkv, 128}, x.options());
  G64Args g{reinterpret_cast<const unsigned short*>(x.data_ptr()), reinterpret_cast<const unsigned short*>(w.data_ptr()),
            reinterpret_cast<unsigned short*>(q.data_ptr()), x.stride(0), K, 0,
            (int)T, (int)N, (int)K, (int)(T / TM), (int)(N / TN), 0, 1, 0, nullptr, nullptr};
  g.out2 = reinterpret_cast<unsigned short*>(k.data_ptr());
  g.out3 = reinterpret_cast<unsigned short*>(v.data_ptr());
  g.cosT = cosT.data_ptr<float>();
  g.sinT = sinT.data_ptr<float>();
  g.pos = has_pos ? pos->data_ptr<int>() : nullptr;
  g.nq = (int)nq;
  g.nkv = (int)nkv;
  g.seq = (int)std::max<int64_t>(seq, 1);
  // tail split (config / 1000, as gemm64_ex) on the 4-wave kernels, whose split items store fp32
  // partials that gemm64_split_reduce rotates; the 8-wave kernel takes whole tiles only
  plan_split(g, (config / 100) % 10 >= 3 ? (int)(config / 1000) : 1);
  at::Tensor ws;
  if (g.splits > 1) {
    ws = at::empty({(long)(g.tiles_m * g.tiles_n - g.n_main) * g.splits * TM * TN}, x.options().dtype(at::kFloat));
    g.ws = ws.data_ptr<float>();
  }
  launch<false, false, EPI_ROPE_QKV>(g, (int)(config % 1000));
  return {q, k, v};
}

// Gate/up projection storing gu [T, 2F] and act = silu(g) * u [T, F] (training forward).
std::tuple<at::Tensor, at::Tensor> gemm64_up_swiglu(const at::Tensor& x, const at::Tensor& w, int64_t config) {
  LLMCTL_CHECK(x.dim() == 2 && w.dim() == 2 && x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16 &&
                   x.is_cuda() && w.is_cuda() && x.stride(1) == 1 && w.is_contiguous(),
               "gemm64_up_swiglu: bf16 GPU x [T, K] (unit inner stride), contiguous W_up [2F, K]");
  const long T = x.size(0), K = x.size(1), F = w.size(0) / 2;
  LLMCTL_CHECK(w.size(1) == K && w.size(0) == 2 * F, "gemm64_up_swiglu: W_up must be [2F, K]");
  LLMCTL_CHECK(T % TM == 0 && F % (TN / 2) == 0 && K % (2 * TK) == 0 && K > 0,
               "gemm64_up_swiglu: T % 256, F % 128, K % 128 (got ", T, "x", F, "x", K, ")");
  LLMCTL_CHECK(x.stride(0) % 8 == 0 && (reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0 &&
                   (long)TM * x.stride(0) * 2 < (1L << 31) && (long)TN * K * 2 < (1L << 31) &&
                   (2 * F) * K * 2 < (1L << 31),
               "gemm64_up_swiglu: 16-byte aligned rows / 32-bit offsets");
  const c10::DeviceGuard dg(x.device());
  auto gu = at::empty({T, 2 * F}, x.options());
  auto act = at::empty({T, F}, x.options());
  G64Args g{reinterpret_cast<const unsigned short*>(x.data_ptr()), reinterpret_cast<const unsigned short*>(w.data_ptr()),
            reinterpret_cast<unsigned short*>(gu.data_ptr()), x.stride(0), K, 2 * F,
            (int)T, (int)F, (int)K, (int)(T / TM), (int)(F / (TN / 2)), 0, 1, 0, nullptr, nullptr};
  g.out2 = reinterpret_cast<unsigned short*>(act.data_ptr());
  plan_split(g, 1);
  launch<false, false, EPI_UP_SWIGLU>(g, (int)(config % 1000));
  return {gu, act};
}

// Row-scaled projection (serving prefill, RMSNorm folded in): y = (x · w^T) * rstd[:, None] in bf16,
// x [M, K] (M % 256), w [N, K] (N % 256) with the norm weight folded into its K columns.
at::Tensor gemm64_rs(const at::Tensor& x, const at::Tensor& w, const at::Tensor& rstd, int64_t config) {
  LLMCTL_CHECK(x.dim() == 2 && w.dim() == 2 && x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16 &&
                   x.is_cuda() && w.is_cuda() && x.stride(1) == 1 && w.is_contiguous(),
               "gemm64_rs: bf16 GPU x [M, K] (unit inner stride), contiguous w [N, K]");
  const long M = x.size(0), K = x.size(1), N = w.size(0);
  LLMCTL_CHECK(w.size(1) == K && gemm64_supported(M, N, K) && K >= 4 * TK,
               "gemm64_rs: M, N multiples of 256, K of 128 and >= 256 (got ", M, "x", N, "x", K, ")");
  LLMCTL_CHECK(x.stride(0) % 8 == 0 && (reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(w.data_ptr()) & 15) == 0 && (long)TM * x.stride(0) * 2 < (1L << 31) &&
                   (long)TN * K * 2 < (1L << 31),
               "gemm64_rs: 16-byte aligned rows / 32-bit offsets");
  check_rstd(rstd, M, "gemm64_rs");
  const c10::DeviceGuard dg(x.device());
  auto y = at::empty({M, N}, x.options());
  G64Args g{reinterpret_cast<const unsigned short*>(x.data_ptr()), reinterpret_cast<const unsigned short*>(w.data_ptr()),
            reinterpret_cast<unsigned short*>(y.data_ptr()), x.stride(0), K, N,
            (int)M, (int)N, (int)K, (int)(M / TM), (int)(N / TN), 0, 1, 0, nullptr, nullptr};
  g.rs = rstd.data_ptr<float>();
  const int cfg = persistent_config(config);
  plan_split(g, cfg / 1000);
  at::Tensor ws;
  if (g.splits > 1) {
    ws = at::empty({(long)(g.tiles_m * g.tiles_n - g.n_main) * g.splits * TM * TN}, x.options().dtype(at::kFloat));
    g.ws = ws.data_ptr<float>();
  }
  launch<false, false, EPI_STORE, true>(g, cfg % 1000);
  return y;
}

TORCH_LIBRARY_IMPL(llmctl, CUDA, m) {
  m.impl("gemm64_rs", &gemm64_rs);
  m.impl("gemm64_qkv_rope", &gemm64_qkv_rope);
  m.impl("gemm64_up_swiglu", &gemm64_up_swiglu);
  m.impl("gemm64_swiglu_fwd", &gemm64_swiglu_fwd);
  m.impl("gemm64_ex", &gemm64_ex);
  m.impl("gemm64_swiglu_dgrad", &gemm64_swiglu_dgrad);
  m.impl("gemm64_wgrad_swiglu", &gemm64_wgrad_swiglu);
}

}  // namespace llmctl
