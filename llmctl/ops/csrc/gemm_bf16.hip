// bf16 MFMA GEMM family for the projection layers (gfx950) + an HBM copy kernel.
//
//   C[M,N] (+)= sum_k A(m,k) * B(n,k)        fp32 accumulate, bf16 in/out
//
// Each operand is read either "K-contiguous" (A stored [M][K], B stored [N][K]) or
// "K-major" (A stored [K][M], B stored [K][N]) — the template flags AT / BT.  That one kernel
// covers all three products of a linear layer y = x W^T without any transpose pass:
//   forward  y  = x  W^T :  A = x  [T][in]    B = W  [out][in]          (AT=0, BT=0)
//   dgrad    dx = dy W   :  A = dy [T][out]   B(n=in,k=out) = W[out][in] (AT=0, BT=1)
//   wgrad    dW = dy^T x :  A(m=out,k=t)=dy[t][out], B(n=in,k=t)=x[t][in] (AT=1, BT=1)
// hipBLASLt's best kernels for the two K-major cases run at ~1.05 PF (wgrad) / ~1.3 PF
// (dgrad) on the GPT-7B shapes (profiles/bench_r1_*); here the K-major image is transposed
// for free by ds_read_b64_tr_b16 on the LDS read.
//
// Structure (CDNA guide §5):
//   * 256x256 workgroup tile, 8 waves (2 along M x 4 along N), each wave owns a 128x64 output
//     block = 8x4 tiles of mfma_f32_16x16x32_bf16 (128 accumulator VGPRs).
//   * K is staged in 32-deep tiles through a 4-slot LDS ring (4 x 32 KB: A image + B image),
//     global -> LDS by global_load_lds_dwordx4 (16 B/lane, no VGPR round trip), prefetch
//     distance 3 tiles.  Ablations of the first 2-slot/BK=64 version showed the kernel was
//     bound by the latency of the one tile in flight (no-MFMA build ran at 87% of the full
//     kernel's time); three tiles in flight keep the load path streaming.
//   * swizzles applied on the per-lane SOURCE address so the lane-linear DMA image is
//     bank-conflict free for the fragment reads (rule 21; SQ_LDS_BANK_CONFLICT = 0 measured).
//   * 2 phases per K-tile: {ds_read fragments; s_barrier; lgkmcnt(0); 16 MFMA; s_barrier}.
//     The two wave groups (waves 0-3 / 4-7, one of each per SIMD) run one barrier apart, so
//     one group's LDS reads overlap the other group's MFMAs (ping-pong).  Raw s_barrier only
//     and counted vmcnt, so the DMA stays in flight across barriers.
//   * XCD-aware bijective block remap + grouped tile order (4 tile-rows per group) so the
//     ~32 concurrently resident tiles of one XCD share A/B panels in that XCD's L2.
//   * Output tiles are computed transposed (B fragment as the MFMA row operand) so each lane
//     holds 4 consecutive output columns: 8-byte stores / read-modify-writes.
#include "attn_common.h"

namespace llmctl {
using namespace attn;
namespace {

using f32x4_t = __attribute__((ext_vector_type(4))) float;
using s2_t = __attribute__((ext_vector_type(2))) unsigned int;

constexpr int TM = 256, TN = 256, TK = 32;
constexpr int IMG = TM * TK * 2;  // 16 KB per operand image
constexpr int SLOT = 2 * IMG;     // A + B = 32 KB
constexpr int NSLOT = 4;
constexpr int NTHR = 512;
constexpr int PIECES = IMG / (NTHR * 16);  // DMA instructions per operand per thread (2)

struct GemmArgs {
  const unsigned short* a;
  const unsigned short* b;
  unsigned short* c;
  long lda, ldb, ldc;
  int M, N, K;
  int tiles_m, tiles_n;
};

__device__ __forceinline__ f32x4_t mfma16(bf16x8_t a, bf16x8_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// LDS DMA (global_load_lds_dwordx4) in inline asm: through the builtin, hipcc treats every
// later ds_read as possibly aliasing the in-flight DMA and drains vmcnt(0) before it, which
// serialises the prefetch with this tile's reads.  Here the ordering is ours: counted
// s_waitcnt vmcnt + s_barrier before a staged slot is read (see the K loop).
__device__ __forceinline__ void glds16(const unsigned short* g, unsigned lds_byte) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(lds_byte) : "memory");
}

// Same DMA through a buffer resource (SGPR V# + 32-bit per-lane byte offset + SGPR k-offset):
// half the per-lane address bytes of the 64-bit flat form.
using i32x4_t = __attribute__((ext_vector_type(4))) int;
__device__ __forceinline__ i32x4_t make_rsrc(const void* base) {
  const unsigned long a = (unsigned long)base;
  i32x4_t r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(a & 0xffffffffu));
  r[1] = __builtin_amdgcn_readfirstlane((int)((a >> 32) & 0xffff));
  r[2] = -1;          // num_records: no clamping (offsets are validated on the host)
  r[3] = 0x00020000;  // raw buffer, 32-bit data format
  return r;
}
__device__ __forceinline__ void bdma16(i32x4_t rsrc, unsigned voff, unsigned soff, unsigned lds_byte) {
  asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(voff), "s"(rsrc),
               "s"(soff), "s"(lds_byte)
               : "memory");
}

// ---- LDS images (one 32-deep K-tile) -------------------------------------------------------
// row image  ("K-contiguous" operand): [256 rows][32 k], 64-B rows, 16-B chunk c -> c ^ fr(row)
//   fr(row) = F[(row>>2)&3] with F = {0,2,3,1}: each ds_read_b128 lane group
//   ({0-3,12-15,20-27}, {4-11,16-19,28-31}, ... : rows 0-3,12-15 at chunk g, rows 4-11 at g+1)
//   lands on 16 distinct 16-B bank slots.
// tr image   ("K-major" operand): [32 k][256 cols], 512-B rows, 32-B segment s -> s ^ ftr(k)
//   ftr(k) = (k&3) | ((k>>3)&1)<<2 : the 8 k-rows of a 32-lane ds_read_b64_tr_b16 half
//   (k = 8g+q, g in {0,1}, q in 0..3) land on 8 distinct 32-B slots.
__device__ __forceinline__ int fr(int row) { return (0x78 >> (2 * ((row >> 2) & 3))) & 3; }
__device__ __forceinline__ int ftr(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }

// Per-thread staging offsets (elements, relative to the operand's tile origin at k0 = 0).
// DMA instruction i of wave w fills image chunks [i*512 + w*64, +64), lane-linear.
template <bool T>
__device__ __forceinline__ long stage_off(int i, int tid, long ld) {
  const int c = i * NTHR + tid;
  if constexpr (!T) {
    const int row = c >> 2, cs = c & 3;
    return (long)row * ld + (cs ^ fr(row)) * 8;
  } else {
    const int k = c >> 5, cs = c & 31;
    return (long)k * ld + (cs ^ (ftr(k) << 1)) * 8;
  }
}

// Fragment of a 16-row (or 16-col for tr) x 32-k block: lane l holds X(r0 + (l&15), 8(l>>4) + j)
template <bool T>
__device__ __forceinline__ bf16x8_t frag(const unsigned char* img, int r0, int lane) {
  const int g = lane >> 4, i16 = lane & 15;
  if constexpr (!T) {
    const int row = r0 + i16;
    return *reinterpret_cast<const bf16x8_t*>(img + row * 64 + ((g ^ fr(i16)) << 4));
  } else {
    const int q = i16 >> 2, p = i16 & 3;
    const int k1 = 8 * g + q;
    const int seg = (r0 >> 4) ^ (q | ((g & 1) << 2));
    const int off = k1 * 512 + ((2 * seg + (p >> 1)) << 4) + (p & 1) * 8;
    s4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + off));
    s4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + off + 4 * 512));
    s8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8_t, v);
  }
}

__device__ __forceinline__ void bar() { __builtin_amdgcn_s_barrier(); }

template <int N>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
}

template <bool AT, bool BT, bool ACC, int V>
__global__ __launch_bounds__(NTHR, 1) void gemm256_kernel(GemmArgs args) {
  // V: schedule variant bits (A/B'd by tools/gemm_variants.py)
  //   1: issue a K-tile's whole DMA (A and B) in phase a instead of A in phase a, B in phase b
  //   2: compiler-counted lgkmcnt before the MFMAs instead of an explicit lgkmcnt(0) drain
  //   4: no s_setprio around the MFMA clusters
  //   16/32/48: tile-order group of 8 / 1 / 16 tile-rows instead of 4
  //   64: skew each tile's K start by (tile % 8) K-tiles (wrapping), so co-resident tiles
  //       stream different lines at any instant
  constexpr bool ONE = V & 1;
  constexpr int GROUP = (V & 48) == 16 ? 8 : (V & 48) == 32 ? 1 : (V & 48) == 48 ? 16 : 4;
  constexpr bool SKEW = V & 64;
  constexpr bool BUF = V & 128;  // 128: buffer_load ... lds DMA instead of global_load_lds
  constexpr bool COUNTED = V & 2;
  constexpr bool PRIO = !(V & 4);
  // timing ablations (results wrong): 512 no MFMA, 1024 no fragment reads
  constexpr bool NOMFMA = V & 512, NOREAD = V & 1024;
  constexpr int NS = (V & 256) ? 5 : NSLOT;  // 256: 5-slot ring (all 160 KB of LDS), distance 4
  constexpr int DIST = NS - 1;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[NS * SLOT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;

  // ---- tile selection: XCD-bijective remap, then grouped (4 tile-rows) order
  const int nwg = gridDim.x, bid = blockIdx.x;
  int wg = bid;
  {
    const int q = nwg / 8, rem = nwg % 8, x = bid % 8;
    wg = (x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q) + bid / 8;
  }
  const int per_group = GROUP * args.tiles_n;
  const int grp = wg / per_group;
  const int gsz = min(GROUP, args.tiles_m - grp * GROUP);
  const int inner = wg - grp * per_group;
  const int tm = grp * GROUP + inner % gsz;
  const int tn = inner / gsz;

  const long lda = args.lda, ldb = args.ldb;
  const unsigned short* Ab = AT ? args.a + (long)tm * TM : args.a + (long)tm * TM * lda;
  const unsigned short* Bb = BT ? args.b + (long)tn * TN : args.b + (long)tn * TN * ldb;
  const long a_kstep = AT ? (long)TK * lda : TK;
  const long b_kstep = BT ? (long)TK * ldb : TK;
  const int KT = args.K / TK;
  const int skew = SKEW ? (wg & 7) % KT : 0;
  auto phys = [&](int kt) { int p = kt + skew; return p >= KT ? p - KT : p; };
  long aoff[PIECES], boff[PIECES];
#pragma unroll
  for (int i = 0; i < PIECES; ++i) {
    aoff[i] = stage_off<AT>(i, tid, lda);
    boff[i] = stage_off<BT>(i, tid, ldb);
  }
  // wave-uniform LDS byte address of this wave's first DMA chunk
  const unsigned lds0 =
      __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)smem) +
      wave * 64 * 16;
  const i32x4_t ra_rs = make_rsrc(Ab), rb_rs = make_rsrc(Bb);
  unsigned avo[PIECES], bvo[PIECES];
#pragma unroll
  for (int i = 0; i < PIECES; ++i) {
    avo[i] = (unsigned)(aoff[i] * 2);
    bvo[i] = (unsigned)(boff[i] * 2);
  }
  auto stage_a = [&](int kt) {  // A image of K-tile kt -> slot kt % 4
    const unsigned l = lds0 + (kt % NS) * SLOT;
    if constexpr (BUF) {
      const unsigned so = __builtin_amdgcn_readfirstlane((unsigned)(phys(kt) * a_kstep * 2));
#pragma unroll
      for (int i = 0; i < PIECES; ++i) bdma16(ra_rs, avo[i], so, l + i * NTHR * 16);
    } else {
#pragma unroll
      for (int i = 0; i < PIECES; ++i) glds16(Ab + phys(kt) * a_kstep + aoff[i], l + i * NTHR * 16);
    }
  };
  auto stage_b = [&](int kt) {
    const unsigned l = lds0 + (kt % NS) * SLOT + IMG;
    if constexpr (BUF) {
      const unsigned so = __builtin_amdgcn_readfirstlane((unsigned)(phys(kt) * b_kstep * 2));
#pragma unroll
      for (int i = 0; i < PIECES; ++i) bdma16(rb_rs, bvo[i], so, l + i * NTHR * 16);
    } else {
#pragma unroll
      for (int i = 0; i < PIECES; ++i) glds16(Bb + phys(kt) * b_kstep + boff[i], l + i * NTHR * 16);
    }
  };
  auto pre_mfma = [&]() {
    if constexpr (!COUNTED) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
  };
  auto post_mfma = [&]() {
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
  };

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int am0 = wr * 128;  // this wave's rows in the A image
  const int bn0 = wc * 64;   // this wave's rows in the B image

  // prologue: K-tiles 0, 1, 2 in flight; wait for tile 0
  {
#pragma unroll
    for (int i = 0; i < DIST; ++i)
      if (i < KT) { stage_a(i); stage_b(i); }
    // wait for tile 0: the younger tiles 1..min(DIST,KT)-1 may stay in flight (4 pieces each)
    const int younger = min(DIST, KT) - 1;
    if (younger >= 3) wait_vm<12>();
    else if (younger == 2) wait_vm<8>();
    else if (younger == 1) wait_vm<4>();
    else wait_vm<0>();
  }
  bar();
  if (wr == 1) bar();  // wave group 1 runs one barrier behind group 0 (ping-pong)

  bf16x8_t af[4], bfr[4];
  for (int kt = 0; kt < KT; ++kt) {
    const unsigned char* sa = smem + (kt % NS) * SLOT;
    const unsigned char* sb = sa + IMG;
    // K-tile kt+DIST goes to the slot last read by K-tile kt-1 (retired before its phase-b MFMAs)
    const bool pf = kt + DIST < KT;
    // ---- phase a: m-tiles 0..3 x n-tiles 0..3
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (!NOREAD || kt == 0) af[i] = frag<AT>(sa, am0 + 16 * i, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (!NOREAD || kt == 0) bfr[j] = frag<BT>(sb, bn0 + 16 * j, lane);
    bar();
    if (pf) {
      stage_a(kt + DIST);
      if constexpr (ONE) stage_b(kt + DIST);
    }
    pre_mfma();
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if constexpr (NOMFMA) asm volatile("" ::"v"(bfr[j]), "v"(af[i]));
        else acc[i][j] = mfma16(bfr[j], af[i], acc[i][j]);
      }
    post_mfma();
    bar();
    // ---- phase b: m-tiles 4..7 (B fragments reused); K-tile kt+1 must have landed before
    //      this phase's first barrier (both wave groups read it right after the next one)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (!NOREAD || kt == 0) af[i] = frag<AT>(sa, am0 + 64 + 16 * i, lane);
    // outstanding DMA pieces younger than K-tile kt+1's: tile kt+2 (4) + tile kt+3's A (2)
    {
      // pieces younger than K-tile kt+1's: tiles kt+2 .. kt+DIST-1 (4 each) + tile kt+DIST's
      // A (2; or A+B = 4 with ONE) issued in phase a
      const int full = min(kt + DIST, KT) - (kt + 2);  // whole younger tiles already issued
      if (kt + 1 < KT) {
        if (kt + DIST < KT) {
          if constexpr (DIST == 4) {
            if constexpr (ONE) wait_vm<12>();
            else wait_vm<10>();
          } else {
            if constexpr (ONE) wait_vm<8>();
            else wait_vm<6>();
          }
        } else if (full >= 2) {
          wait_vm<8>();
        } else if (full == 1) {
          wait_vm<4>();
        } else {
          wait_vm<0>();
        }
      }
    }
    bar();
    if (!ONE && pf) stage_b(kt + DIST);
    pre_mfma();
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if constexpr (NOMFMA) asm volatile("" ::"v"(bfr[j]), "v"(af[i]));
        else acc[4 + i][j] = mfma16(bfr[j], af[i], acc[4 + i][j]);
      }
    post_mfma();
    bar();
  }
  if (wr == 0) bar();  // re-align the barrier count of the two groups

  // ---- epilogue: lane holds C[m = .. + (l&15)][n = .. + 4(l>>4) + r], r = 0..3
  const int g = lane >> 4, i16 = lane & 15;
  unsigned short* Cb = args.c + (long)(tm * TM + am0 + i16) * args.ldc + tn * TN + bn0 + 4 * g;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      unsigned short* p = Cb + (long)(16 * i) * args.ldc + 16 * j;
      f32x4_t v = acc[i][j];
      if constexpr (ACC) {
        const s2_t old = *reinterpret_cast<const s2_t*>(p);
        v[0] += bf2f(old[0] & 0xffff);
        v[1] += bf2f(old[0] >> 16);
        v[2] += bf2f(old[1] & 0xffff);
        v[3] += bf2f(old[1] >> 16);
      }
      s2_t o;
      o[0] = (unsigned)f2bf(v[0]) | ((unsigned)f2bf(v[1]) << 16);
      o[1] = (unsigned)f2bf(v[2]) | ((unsigned)f2bf(v[3]) << 16);
      *reinterpret_cast<s2_t*>(p) = o;
    }
  }
}

__global__ __launch_bounds__(256) void copy_kernel(const uint4* __restrict__ s, uint4* __restrict__ d, long n16) {
  const long stride = (long)gridDim.x * 256;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) d[i] = s[i];
}

template <bool AT, bool BT, bool ACC, int V>
void launch_v(const GemmArgs& g) {
  hipLaunchKernelGGL((gemm256_kernel<AT, BT, ACC, V>), dim3(g.tiles_m * g.tiles_n), dim3(NTHR), 0, stream(), g);
}

// measured best schedule per layout (tools/gemm_variants.py, 7B shapes): buffer-DMA, with the
// whole K-tile DMA in phase a for wgrad (AT && BT) and compiler-counted lgkmcnt otherwise
constexpr int kDefaultVariantW = 129, kDefaultVariant = 130;

template <bool AT, bool BT, bool ACC>
void launch(const GemmArgs& g, int variant) {
  switch (variant < 0 ? (AT && BT ? kDefaultVariantW : kDefaultVariant) : variant) {
    case 0: launch_v<AT, BT, ACC, 0>(g); break;
    case 1: launch_v<AT, BT, ACC, 1>(g); break;
    case 2: launch_v<AT, BT, ACC, 2>(g); break;
    case 3: launch_v<AT, BT, ACC, 3>(g); break;
    case 4: launch_v<AT, BT, ACC, 4>(g); break;
    case 5: launch_v<AT, BT, ACC, 5>(g); break;
    case 6: launch_v<AT, BT, ACC, 6>(g); break;
    case 7: launch_v<AT, BT, ACC, 7>(g); break;
    case 16: launch_v<AT, BT, ACC, 16>(g); break;
    case 32: launch_v<AT, BT, ACC, 32>(g); break;
    case 48: launch_v<AT, BT, ACC, 48>(g); break;
    case 64: launch_v<AT, BT, ACC, 64>(g); break;
    case 80: launch_v<AT, BT, ACC, 80>(g); break;
    case 128: launch_v<AT, BT, ACC, 128>(g); break;
    case 130: launch_v<AT, BT, ACC, 130>(g); break;
    case 129: launch_v<AT, BT, ACC, 129>(g); break;
    case 384: launch_v<AT, BT, ACC, 384>(g); break;
    case 640: launch_v<AT, BT, ACC, 640>(g); break;     // 128 | NOMFMA
    case 1664: launch_v<AT, BT, ACC, 1664>(g); break;   // 128 | NOMFMA | NOREAD
    case 1152: launch_v<AT, BT, ACC, 1152>(g); break;   // 128 | NOREAD
    case 385: launch_v<AT, BT, ACC, 385>(g); break;
    case 386: launch_v<AT, BT, ACC, 386>(g); break;
    default: launch_v<AT, BT, ACC, 14>(g); break;
  }
}

}  // namespace

// out[M,N] (+)= A·B^T with operand storage selected by at / bt (see header).  Shapes are the
// *logical* M, N, K; a / b are 2-D row-major tensors ([M,K] or [K,M]; [N,K] or [K,N]).
void gemm_ex(const at::Tensor& a, const at::Tensor& b, at::Tensor& out, bool at_, bool bt_, bool accumulate,
             int64_t variant) {
  LLMCTL_CHECK(a.dim() == 2 && b.dim() == 2 && out.dim() == 2, "gemm_ex: 2-D operands");
  LLMCTL_CHECK(a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16 &&
                   out.scalar_type() == at::kBFloat16, "gemm_ex: bf16 operands");
  LLMCTL_CHECK(a.stride(1) == 1 && b.stride(1) == 1 && out.stride(1) == 1, "gemm_ex: unit inner stride");
  const long M = at_ ? a.size(1) : a.size(0);
  const long K = at_ ? a.size(0) : a.size(1);
  const long N = bt_ ? b.size(1) : b.size(0);
  const long Kb = bt_ ? b.size(0) : b.size(1);
  LLMCTL_CHECK(K == Kb, "gemm_ex: K mismatch (", K, " vs ", Kb, ")");
  LLMCTL_CHECK(out.size(0) == M && out.size(1) == N, "gemm_ex: out must be [M,N]");
  LLMCTL_CHECK(M % TM == 0 && N % TN == 0 && K % TK == 0 && K >= TK, "gemm_ex: M,N multiples of 256, K of 32 (got ",
               M, "x", N, "x", K, ")");
  LLMCTL_CHECK(a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0 && out.stride(0) % 4 == 0 &&
                   (reinterpret_cast<uintptr_t>(a.data_ptr()) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(b.data_ptr()) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(out.data_ptr()) & 7) == 0,
               "gemm_ex: 16-byte aligned operand rows");
  const c10::DeviceGuard dg(a.device());
  GemmArgs g{bf_ptr(a), bf_ptr(b), bf_mut(out), a.stride(0), b.stride(0), out.stride(0),
             (int)M, (int)N, (int)K, (int)(M / TM), (int)(N / TN)};
  const int sel = (at_ ? 4 : 0) | (bt_ ? 2 : 0) | (accumulate ? 1 : 0);
  switch (sel) {
    case 0: launch<false, false, false>(g, (int)variant); break;
    case 1: launch<false, false, true>(g, (int)variant); break;
    case 2: launch<false, true, false>(g, (int)variant); break;
    case 3: launch<false, true, true>(g, (int)variant); break;
    case 4: launch<true, false, false>(g, (int)variant); break;
    case 5: launch<true, false, true>(g, (int)variant); break;
    case 6: launch<true, true, false>(g, (int)variant); break;
    default: launch<true, true, true>(g, (int)variant); break;
  }
}

at::Tensor gemm_bf16(const at::Tensor& a, const at::Tensor& b) {
  LLMCTL_CHECK(a.dim() == 2 && b.dim() == 2 && b.size(1) == a.size(1), "gemm_bf16: A[M,K], B[N,K]");
  auto c = at::empty({a.size(0), b.size(0)}, a.options());
  gemm_ex(a.contiguous(), b.contiguous(), c, false, false, false, -1);
  return c;
}

void hbm_copy(const at::Tensor& src, at::Tensor& dst) {
  LLMCTL_CHECK(src.is_contiguous() && dst.is_contiguous() && src.nbytes() == dst.nbytes() && src.nbytes() % 16 == 0,
               "hbm_copy: contiguous, equal size, multiple of 16 bytes");
  const c10::DeviceGuard g(src.device());
  const long n16 = src.nbytes() / 16;
  const int grid = (int)std::min<long>((n16 + 255) / 256, (long)num_cus() * 8);
  hipLaunchKernelGGL(copy_kernel, dim3(grid), dim3(256), 0, stream(), reinterpret_cast<const uint4*>(src.data_ptr()),
                     reinterpret_cast<uint4*>(dst.data_ptr()), n16);
}

TORCH_LIBRARY_IMPL(llmctl, CUDA, m) {
  m.impl("gemm_bf16", &gemm_bf16);
  m.impl("gemm_ex", &gemm_ex);
  m.impl("hbm_copy", &hbm_copy);
}

}  // namespace llmctl
