// EXPERIMENT (not built: llmctl/ops/build.py compiles csrc/*.hip only; to measure it, move it back
// to csrc/ and add "gemm_w4_ex(Tensor a, Tensor b, Tensor(a!) out, bool at, bool bt, bool accumulate,
// int config=4) -> ()" to bindings.cpp; tools/gemm64_bench.py --w4 <configs> runs it).
// Status (round 2, correct on every GPT-7B projection shape, tools/gpu_r2_w4.sh): 1.21-1.42 PF,
// i.e. at or below gemm64 (1.28-1.45 PF) and well below hipBLASLt's forward kernel (1.45-1.63 PF,
// also one wave per SIMD at 256x256x64).  Variants: register-staged operands (0xx: 57 % MFMA busy
// by PMC), two-stage (1xx: no change, so not load latency), LDS-DMA (2xx: +1-3 %), LDS-DMA with
// one filler per MFMA pinned by sched_barrier (3xx: +3-5 % over 2xx).
//
// bf16 MFMA GEMM, 256x256 tile, ONE wave per SIMD (4 waves x 128x128 outputs), register-staged
// 64-deep K-tiles (gfx950).
//
// The 256 accumulators live in AGPRs through inline-asm MFMA batches ("+a" operands, one column
// of 8 MFMAs per statement): with the builtin, hipcc (ROCm 7.2) kept them in VGPRs/AGPRs by turns
// and the main loop carried ~350 v_accvgpr_* moves per 128 MFMAs plus spills.
//
//   C[M,N] (+)= sum_k A(m,k) * B(n,k)        fp32 accumulate, bf16 in/out
//
// Operand storage as in gemm64.hip (AT / BT: K-major operand).
//
// Why this shape (profiles/gemm64_pmc_r2.txt): the 8-wave gemm64 (2 waves/SIMD, 128x64 per
// wave) reads 24 ds_read_b128 per wave per K-tile = 192 KB of LDS per K-tile per CU and holds
// the MFMA pipe ~75 % busy; hipBLASLt's forward kernel on the same shape issues 32 reads per
// wave per K-tile with 4 waves = 128 KB (one wave per SIMD owning 128x128 outputs: 256
// accumulators in AGPRs) and keeps the pipe ~84 % busy.  A wave that is alone on its SIMD
// cannot hide LDS-DMA issue (≈60 cycles per piece among MFMAs, MI355X_MICROARCH.md) behind a
// partner wave, so operands are staged through registers: buffer_load_dwordx4 (cheap issue)
// for K-tile t+2 during K-tile t, ds_write_b128 of K-tile t+1 (swizzle applied on the write),
// all interleaved into the MFMA stream.
//
// Per K-tile t (two 32-deep sub-steps; fragments double-buffered in registers; the register
// stage holds ONE operand of one K-tile = 8 x 16 B per thread):
//   part 1: MFMA(t, k0..31)  | ds_read frags (t, k32..63) | ds_write stage -> B image of t+1,
//           then buffer_load A of K-tile t+2 -> stage
//   LDS barrier (K-tile t+1 complete and visible; every wave done reading K-tile t's buffer)
//   part 2: MFMA(t, k32..63) | ds_read frags (t+1, k0..31) | ds_write stage -> A image of t+2
//           (into K-tile t's buffer, now free), then buffer_load B of t+2 -> stage
// Two K-tile LDS buffers (128 KB); every load has one part (64 MFMAs) to land.
#include "attn_common.h"

namespace llmctl {
using namespace attn;
namespace {

using f32x4_t = __attribute__((ext_vector_type(4))) float;
using s2_t = __attribute__((ext_vector_type(2))) unsigned int;
using i32x4_t = __attribute__((ext_vector_type(4))) int;
template <int V>
using K_ = std::integral_constant<int, V>;

constexpr int TM = 256, TN = 256, TK = 64;
constexpr int NTHR = 256;
constexpr int IMG = TM * TK * 2;  // 32 KB per operand image
constexpr int BUF = 2 * IMG;      // A + B of one K-tile
constexpr int PIECES = IMG / (NTHR * 16);  // 8 x 16 B per thread per operand per K-tile

struct W4Args {
  const unsigned short* a;
  const unsigned short* b;
  unsigned short* c;
  long lda, ldb, ldc;
  int M, N, K;
  int tiles_m, tiles_n;
};

// one output column block j: acc[i][j] += B_j(16 n x 32 k) x A_i(16 m x 32 k), i = 0..7, computed
// transposed (B fragment as the row operand: a lane holds 4 consecutive n).  hipcc pads no wait
// states inside asm: NOP = "s_nop 1" for a VALU-written operand; the LDS-DMA kernel's fragments
// come straight from ds_read (covered by the compiler's lgkmcnt wait; its loops carry no VALU
// writes to them: checked in the ISA) and it runs without.
template <bool NOP = true>
__device__ __forceinline__ void mma_col(f32x4_t& c0, f32x4_t& c1, f32x4_t& c2, f32x4_t& c3, f32x4_t& c4, f32x4_t& c5,
                                        f32x4_t& c6, f32x4_t& c7, bf16x8_t b, const bf16x8_t* a) {
  if constexpr (NOP) asm volatile("s_nop 1");
  asm volatile(
      "v_mfma_f32_16x16x32_bf16 %0, %8, %9, %0\n\t"
      "v_mfma_f32_16x16x32_bf16 %1, %8, %10, %1\n\t"
      "v_mfma_f32_16x16x32_bf16 %2, %8, %11, %2\n\t"
      "v_mfma_f32_16x16x32_bf16 %3, %8, %12, %3\n\t"
      "v_mfma_f32_16x16x32_bf16 %4, %8, %13, %4\n\t"
      "v_mfma_f32_16x16x32_bf16 %5, %8, %14, %5\n\t"
      "v_mfma_f32_16x16x32_bf16 %6, %8, %15, %6\n\t"
      "v_mfma_f32_16x16x32_bf16 %7, %8, %16, %7"
      : "+a"(c0), "+a"(c1), "+a"(c2), "+a"(c3), "+a"(c4), "+a"(c5), "+a"(c6), "+a"(c7)
      : "v"(b), "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]));
}
// 4-pass XDL result -> non-MFMA reader: pad before the epilogue touches the accumulators
__device__ __forceinline__ void acc_fence(f32x4_t& c0, f32x4_t& c1, f32x4_t& c2, f32x4_t& c3, f32x4_t& c4, f32x4_t& c5,
                                          f32x4_t& c6, f32x4_t& c7) {
  asm volatile("s_nop 7\n\ts_nop 7"
               : "+a"(c0), "+a"(c1), "+a"(c2), "+a"(c3), "+a"(c4), "+a"(c5), "+a"(c6), "+a"(c7));
}

// one MFMA on an AGPR accumulator (the unit the interleaved schedules place one filler after)
__device__ __forceinline__ void mma1(f32x4_t& c, bf16x8_t b, bf16x8_t a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(b), "v"(a));
}

// raw buffer resource over the operand tile: no clamping (offsets validated on the host)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, -1, 0x00020000);
}

// ---- LDS images of one K-tile operand (32 KB) ------------------------------------------------
// row image (K-contiguous): [256 rows][64 k], 128-B rows, chunk c at c ^ ((row >> 1) & 7)
// tr image  (K-major):      [64 k][256 cols], 512-B rows, 32-B segment s at s ^ h(k),
//                           h(k) = (k & 3) | ((k >> 3) & 1) << 2
__device__ __forceinline__ int swr(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ int swt(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }

// Staging piece i (0..7) of thread tid covers 16 B of the operand's K-tile image.  The global
// offset is  voff(tid) + i * pstep  (pstep goes into the SGPR soffset) and the LDS offset is
//   row image: row = 32 i + tid / 8, chunk = tid % 8 -> loff(tid) + 4096 i  (swizzle is i-free)
//   tr image:  k = 8 i + tid / 32,   chunk = tid % 32 -> loff(tid, i & 1) + 4096 i
template <bool T>
__device__ __forceinline__ unsigned stage_voff(int tid, long ld) {
  if constexpr (!T) return (unsigned)(((long)(tid >> 3) * ld + (tid & 7) * 8) * 2);
  else return (unsigned)(((long)(tid >> 5) * ld + (tid & 31) * 8) * 2);
}
template <bool T>
__device__ __forceinline__ unsigned stage_pstep(long ld) {  // bytes between pieces i and i+1
  return (unsigned)((T ? 8 : 32) * ld * 2);
}
template <bool T>
__device__ __forceinline__ unsigned stage_loff(int tid, int parity) {
  if constexpr (!T) {
    const int row = tid >> 3, ch = tid & 7;
    return (unsigned)(row * 128 + ((ch ^ swr(row)) << 4));
  } else {
    const int k = 8 * parity + (tid >> 5), ch = tid & 31;
    const int seg = (ch >> 1) ^ swt(k);
    return (unsigned)((tid >> 5) * 512 + seg * 32 + (ch & 1) * 16);
  }
}

template <bool T>
__device__ __forceinline__ bf16x8_t frag(const unsigned char* img, int p0, int ks, int lane) {
  const int g = lane >> 4, i16 = lane & 15;
  if constexpr (!T) {
    const int row = p0 + i16;
    const int c = ks * 4 + g;
    return *reinterpret_cast<const bf16x8_t*>(img + row * 128 + ((c ^ swr(row)) << 4));
  } else {
    const int q = i16 >> 2, p = i16 & 3;
    const int k = ks * 32 + 8 * g + q;
    const int seg = (p0 >> 4) ^ swt(k);
    const int off = k * 512 + seg * 32 + p * 8;
    s4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + off));
    s4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + off + 4 * 512));
    s8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8_t, v);
  }
}

// bf16 store (ACC: added to C) of a wave's 128 x 128 block: lane holds
// C[m = am + 16 i + (l & 15)][n = bn + 16 j + 4 (l >> 4) + r]
template <bool ACC>
__device__ __forceinline__ void w4_store(const W4Args& args, f32x4_t (&acc)[8][8], int tm, int tn, int am, int bn,
                                         int lane) {
  const int g = lane >> 4, i16 = lane & 15;
  unsigned short* Cb = args.c + (long)(tm * TM + am + i16) * args.ldc + tn * TN + bn + 4 * g;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
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

// XCD-bijective block remap + grouped tile order (GROUP tile-rows), as gemm64
template <int GROUP>
__device__ __forceinline__ void w4_tile(const W4Args& args, int& tm, int& tn) {
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q = nwg / 8, rem = nwg % 8, x = bid % 8;
  const int wg = (x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q) + bid / 8;
  const int per_group = GROUP * args.tiles_n;
  const int grp = wg / per_group;
  const int gsz = min(GROUP, args.tiles_m - grp * GROUP);
  const int inner = wg - grp * per_group;
  tm = grp * GROUP + inner % gsz;
  tn = inner / gsz;
}

template <bool AT, bool BT, bool ACC, int GROUP, bool DEEP>
__global__ __launch_bounds__(NTHR, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm_w4_kernel(W4Args args) {
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;

  const int nwg = gridDim.x, bid = blockIdx.x;
  int wg;
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
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(Ab), rb = make_rsrc(Bb);
  const unsigned a_kstep = AT ? (unsigned)(TK * lda * 2) : (unsigned)(TK * 2);
  const unsigned b_kstep = BT ? (unsigned)(TK * ldb * 2) : (unsigned)(TK * 2);
  const int KT = args.K / TK;

  const unsigned avo = stage_voff<AT>(tid, lda), bvo = stage_voff<BT>(tid, ldb);
  const unsigned aps = stage_pstep<AT>(lda), bps = stage_pstep<BT>(ldb);
  const unsigned alo0 = stage_loff<AT>(tid, 0), alo1 = stage_loff<AT>(tid, 1);
  const unsigned blo0 = stage_loff<BT>(tid, 0), blo1 = stage_loff<BT>(tid, 1);
  // register stage: DEEP = one stage per operand (every load has two parts, ~2 x 64 MFMAs, to
  // land); otherwise one shared stage (one part)
  i32x4_t st0[PIECES], st1[PIECES];
  auto& sA = st0;
  auto& sB = DEEP ? st1 : st0;

  // one operand of K-tile t (clamped: past-the-end loads re-read the last tile) -> its stage
  auto gload = [&](auto op_c, int t) {
    constexpr bool isA = decltype(op_c)::value == 0;
    auto& st = isA ? sA : sB;
    const int tc = t < KT ? t : KT - 1;
    const unsigned so0 = (unsigned)tc * (isA ? a_kstep : b_kstep);
#pragma unroll
    for (int i = 0; i < PIECES; ++i) {
      const int so = __builtin_amdgcn_readfirstlane((int)(so0 + i * (isA ? aps : bps)));
      st[i] = __builtin_amdgcn_raw_buffer_load_b128(isA ? ra : rb, isA ? avo : bvo, so, 0);
    }
  };
  auto swrite = [&](auto op_c, unsigned char* buf) {  // stage -> that operand's image in buf
    constexpr bool isA = decltype(op_c)::value == 0;
    auto& st = isA ? sA : sB;
    unsigned char* img = buf + (isA ? 0 : IMG);
#pragma unroll
    for (int i = 0; i < PIECES; ++i) {
      const unsigned lo = (i & 1) ? (isA ? alo1 : blo1) : (isA ? alo0 : blo0);
      *reinterpret_cast<i32x4_t*>(img + lo + 4096 * i) = st[i];
    }
  };

  f32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  bf16x8_t fa[2][8], fb[2][8];
  const int am = wr * 128, bn = wc * 128;
  auto rfrags = [&](auto slot_c, const unsigned char* buf, int ks) {
    constexpr int s = decltype(slot_c)::value;
#pragma unroll
    for (int i = 0; i < 8; ++i) fa[s][i] = frag<AT>(buf, am + 16 * i, ks, lane);
#pragma unroll
    for (int j = 0; j < 8; ++j) fb[s][j] = frag<BT>(buf + IMG, bn + 16 * j, ks, lane);
  };

  // One part = the 64 MFMAs of one 32-deep sub-step on fragment slot C, interleaved column by
  // column with: the next sub-step's fragments (slot 1-C, read from rbuf at depth rks; column
  // j's B fragment reuses the register column j's MFMAs just released), one piece of the
  // stage -> wbuf (operand OP) and the reload of that stage piece from K-tile t_load: with one
  // shared stage the OTHER operand (part 1 writes B(t+1) and loads A(t+2); part 2 writes A(t+2)
  // and loads B(t+2)), with DEEP the same one (part 1: B(t+1) / B(t+2); part 2: A(t+2) / A(t+3)).
  auto part = [&](auto c_c, const unsigned char* rbuf, int rks, auto op_c, unsigned char* wbuf, int t_load) {
    constexpr int C = decltype(c_c)::value, N = 1 - C;
    constexpr bool isA = decltype(op_c)::value == 0;
    auto& st = isA ? sA : sB;
    unsigned char* img = wbuf + (isA ? 0 : IMG);
    const int tc = t_load < KT ? t_load : KT - 1;
    constexpr bool ldA = DEEP ? isA : !isA;
    const unsigned so0 = (unsigned)tc * (ldA ? a_kstep : b_kstep);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      mma_col(acc[0][j], acc[1][j], acc[2][j], acc[3][j], acc[4][j], acc[5][j], acc[6][j], acc[7][j], fb[C][j], fa[C]);
      fa[N][j] = frag<AT>(rbuf, am + 16 * j, rks, lane);
      fb[N][j] = frag<BT>(rbuf + IMG, bn + 16 * j, rks, lane);
      const unsigned lo = (j & 1) ? (isA ? alo1 : blo1) : (isA ? alo0 : blo0);
      *reinterpret_cast<i32x4_t*>(img + lo + 4096 * j) = st[j];
      const int so = __builtin_amdgcn_readfirstlane((int)(so0 + j * (ldA ? aps : bps)));
      st[j] = __builtin_amdgcn_raw_buffer_load_b128(ldA ? ra : rb, ldA ? avo : bvo, so, 0);
    }
  };

  // prologue: K-tile 0 -> buffer 0, A(1) -> buffer 1, B(1) in the stage (+ A(2) with DEEP),
  // frags (0, k0)
  gload(K_<0>{}, 0);
  swrite(K_<0>{}, smem);
  gload(K_<1>{}, 0);
  swrite(K_<1>{}, smem);
  gload(K_<0>{}, 1);
  swrite(K_<0>{}, smem + BUF);
  gload(K_<1>{}, 1);
  if constexpr (DEEP) gload(K_<0>{}, 2);
  lds_sync();
  rfrags(K_<0>{}, smem, 0);

  // K-tile t in buf; nbuf holds K-tile t+1's A image (written in the previous part 2)
  auto ktile = [&](int t, unsigned char* buf, unsigned char* nbuf) {
    // part 1: MFMA(t, k0..31) | frags (t, k32..63) | B(t+1) stage -> nbuf | load A(t+2)
    part(K_<0>{}, buf, 1, K_<1>{}, nbuf, t + 2);
    lds_sync();  // K-tile t+1 complete and visible; every wave is done reading buf
    // part 2: MFMA(t, k32..63) | frags (t+1, k0..31) | A(t+2) stage -> buf | load B(t+2) / A(t+3)
    part(K_<1>{}, nbuf, 0, K_<0>{}, buf, DEEP ? t + 3 : t + 2);
  };

  // one K-tile per iteration (buffers picked by parity at run time): a 2x-unrolled body gets
  // different accumulator registers in its two copies and hipcc then permutes all 256 AGPRs
  // with v_accvgpr_mov at every iteration
  for (int t = 0; t < KT; ++t) {
    unsigned char* buf = smem + (t & 1) * BUF;
    ktile(t, buf, smem + ((t + 1) & 1) * BUF);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the clamped tail loads
#pragma unroll
  for (int j = 0; j < 8; ++j)
    acc_fence(acc[0][j], acc[1][j], acc[2][j], acc[3][j], acc[4][j], acc[5][j], acc[6][j], acc[7][j]);

  w4_store<ACC>(args, acc, tm, tn, am, bn, lane);
}


// ---- LDS-DMA variant (config 200+) -----------------------------------------------------------
// Same images, fragments and MFMA batches; the K-tile is filled by LDS-DMA (buffer_load_dwordx4
// ... lds: 1 KiB per wave-instruction, lane-linear, the image swizzle applied to the SOURCE), so
// no stage registers and no ds_write.  Per K-tile t (buffers by parity):
//   part 1: MFMA(t, k0..31) | frags (t, k32..63)
//   vmcnt(0) (this wave's DMA of t+1 landed) + barrier (everyone's; buffer t fully read)
//   part 2: MFMA(t, k32..63) | frags (t+1, k0..31) | DMA of K-tile t+2 -> buffer t (2 per column)
// Every DMA has part 2 + part 1 (~128 MFMAs) to land.
//
// DMA piece p (0..31) of an operand image = image bytes [1024 p, +1024); wave w issues
// p = 4 i + w, i = 0..7 (A and B one each per column).  Source of lane l:
//   row image: row = 8 p + (l >> 3), stored chunk l & 7 = logical chunk ^ swr(row)
//   tr image:  k = 2 p + (l >> 5), stored segment (l & 31) >> 1 = logical segment ^ swt(k)
// i enters as 32 i rows (row image: swr unchanged) or 8 i k-rows (tr image: swt's bit 2 = i & 1),
// so the per-lane part is one VGPR (two for a tr image, by i parity) and the rest is soffset.
template <bool T>
__device__ __forceinline__ unsigned dma_voff(int w, int lane, int parity, long ld) {
  if constexpr (!T) {
    const int row = 8 * w + (lane >> 3);
    const int c = (lane & 7) ^ swr(row);
    return (unsigned)(((long)row * ld + c * 8) * 2);
  } else {
    const int k = 2 * w + (lane >> 5);
    const int kk = k + 8 * parity;  // swt of the piece's real k-row
    const int seg = ((lane & 31) >> 1) ^ swt(kk);
    return (unsigned)(((long)k * ld + seg * 16 + (lane & 1) * 8) * 2);
  }
}
template <bool T>
__device__ __forceinline__ unsigned dma_istep(long ld) {  // source bytes between pieces i and i+1
  return (unsigned)((T ? 8 : 32) * ld * 2);
}
__device__ __forceinline__ void dma16(i32x4_t rsrc, unsigned voff, unsigned soff, unsigned lds_byte) {
  asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(voff), "s"(rsrc),
               "s"(soff), "s"(lds_byte)
               : "memory");
}
__device__ __forceinline__ i32x4_t raw_rsrc(const void* base) {
  const unsigned long a = (unsigned long)base;
  i32x4_t r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(a & 0xffffffffu));
  r[1] = __builtin_amdgcn_readfirstlane((int)((a >> 32) & 0xffff));
  r[2] = -1;          // no clamping (offsets validated on the host)
  r[3] = 0x00020000;  // raw buffer, 32-bit data format
  return r;
}

template <bool AT, bool BT, bool ACC, int GROUP, bool ILV>
__global__ __launch_bounds__(NTHR, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm_w4d_kernel(W4Args args) {
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  int tm, tn;
  w4_tile<GROUP>(args, tm, tn);

  const long lda = args.lda, ldb = args.ldb;
  const unsigned short* Ab = AT ? args.a + (long)tm * TM : args.a + (long)tm * TM * lda;
  const unsigned short* Bb = BT ? args.b + (long)tn * TN : args.b + (long)tn * TN * ldb;
  const i32x4_t ra = raw_rsrc(Ab), rb = raw_rsrc(Bb);
  const unsigned a_kstep = AT ? (unsigned)(TK * lda * 2) : (unsigned)(TK * 2);
  const unsigned b_kstep = BT ? (unsigned)(TK * ldb * 2) : (unsigned)(TK * 2);
  const unsigned a_is = dma_istep<AT>(lda), b_is = dma_istep<BT>(ldb);
  const int KT = args.K / TK;
  const unsigned va0 = dma_voff<AT>(wave, lane, 0, lda), va1 = dma_voff<AT>(wave, lane, 1, lda);
  const unsigned vb0 = dma_voff<BT>(wave, lane, 0, ldb), vb1 = dma_voff<BT>(wave, lane, 1, ldb);
  const unsigned lds0 = lds_addr(smem) + wave * 1024;

  // pieces i of both operands of K-tile t (clamped) -> buffer t & 1
  auto dma_piece = [&](int t, int i) __attribute__((always_inline)) {
    const unsigned tc = (unsigned)(t < KT ? t : KT - 1);
    const unsigned l = lds0 + (unsigned)((t & 1) * BUF + i * 4096);
    dma16(ra, (i & 1) ? va1 : va0, tc * a_kstep + i * a_is, l);
    dma16(rb, (i & 1) ? vb1 : vb0, tc * b_kstep + i * b_is, l + IMG);
  };

  f32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  bf16x8_t fa[2][8], fb[2][8];
  const int am = wr * 128, bn = wc * 128;

  // prologue: K-tiles 0 and 1 in flight; frags (0, k0..31) once tile 0 landed
#pragma unroll
  for (int i = 0; i < 8; ++i) dma_piece(0, i);
#pragma unroll
  for (int i = 0; i < 8; ++i) dma_piece(1, i);
  vm_wait_n<16>();
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    fa[0][j] = frag<AT>(smem, am + 16 * j, 0, lane);
    fb[0][j] = frag<BT>(smem + IMG, bn + 16 * j, 0, lane);
  }

  // next-slot fragments are read in the first half of each part (4 per column), so their
  // latency is covered before the part boundary's lgkmcnt wait
  if constexpr (!ILV) {
    for (int t = 0; t < KT; ++t) {
      const unsigned char* buf = smem + (t & 1) * BUF;
      const unsigned char* nbuf = smem + ((t + 1) & 1) * BUF;
      // part 1
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        mma_col<false>(acc[0][j], acc[1][j], acc[2][j], acc[3][j], acc[4][j], acc[5][j], acc[6][j], acc[7][j], fb[0][j],
                       fa[0]);
        if (j < 4) {
#pragma unroll
          for (int u = 2 * j; u < 2 * j + 2; ++u) {
            fa[1][u] = frag<AT>(buf, am + 16 * u, 1, lane);
            fb[1][u] = frag<BT>(buf + IMG, bn + 16 * u, 1, lane);
          }
        }
      }
      vm_wait_n<0>();
      lds_sync();
      // part 2
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        mma_col<false>(acc[0][j], acc[1][j], acc[2][j], acc[3][j], acc[4][j], acc[5][j], acc[6][j], acc[7][j], fb[1][j],
                       fa[1]);
        if (j < 4) {
#pragma unroll
          for (int u = 2 * j; u < 2 * j + 2; ++u) {
            fa[0][u] = frag<AT>(nbuf, am + 16 * u, 0, lane);
            fb[0][u] = frag<BT>(nbuf + IMG, bn + 16 * u, 0, lane);
          }
        }
        dma_piece(t + 2, j);
      }
    }
  } else {
    // ILV: one filler after each MFMA, pinned by sched_barrier (a column of 8 MFMAs issued
    // back to back leaves its fillers' issue time exposed: ~40 cycles per column gap):
    //   MFMA slot 0..3 of columns 0..3: next-slot fragment A(2j), B(2j), A(2j+1), B(2j+1)
    //   MFMA slots 4-7 of columns 0..3 in part 2: DMA pieces 2j, 2j+1 of A, then of B (all of
    //   K-tile t+2 in flight by mid-part: ~1.5 parts to land before the next barrier's vmcnt(0))
    auto part = [&](auto c_c, const unsigned char* rb_, int rks, bool dma, int t) __attribute__((always_inline)) {
      constexpr int C = decltype(c_c)::value, N = 1 - C;
      const unsigned tc = (unsigned)(t + 2 < KT ? t + 2 : KT - 1);
      const unsigned lbase = lds0 + (unsigned)(((t + 2) & 1) * BUF);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          mma1(acc[i][j], fb[C][j], fa[C][i]);
          if (j < 4 && i < 4) {
            const int u = 2 * j + (i >> 1);
            if (i & 1) fb[N][u] = frag<BT>(rb_ + IMG, bn + 16 * u, rks, lane);
            else fa[N][u] = frag<AT>(rb_, am + 16 * u, rks, lane);
          }
          if (dma && j < 4 && i >= 4) {  // pieces 2j, 2j+1 of A (slots 4, 5) and B (6, 7)
            const int pc = 2 * j + (i & 1);
            if (i < 6) dma16(ra, (pc & 1) ? va1 : va0, tc * a_kstep + pc * a_is, lbase + pc * 4096);
            else dma16(rb, (pc & 1) ? vb1 : vb0, tc * b_kstep + pc * b_is, lbase + pc * 4096 + IMG);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    };
    for (int t = 0; t < KT; ++t) {
      const unsigned char* buf = smem + (t & 1) * BUF;
      const unsigned char* nbuf = smem + ((t + 1) & 1) * BUF;
      part(K_<0>{}, buf, 1, false, t);
      vm_wait_n<0>();
      lds_sync();
      part(K_<1>{}, nbuf, 0, true, t);
    }
  }
  vm_wait_n<0>();  // the clamped tail pieces
#pragma unroll
  for (int j = 0; j < 8; ++j)
    acc_fence(acc[0][j], acc[1][j], acc[2][j], acc[3][j], acc[4][j], acc[5][j], acc[6][j], acc[7][j]);
  w4_store<ACC>(args, acc, tm, tn, am, bn, lane);
}

// config = group (4 / 8) + 100 * variant (0: register stage, 1: deep register stage, 2: LDS-DMA,
//          3: LDS-DMA with one filler per MFMA)
template <bool AT, bool BT, bool ACC>
void launch(const W4Args& g, int config) {
  const dim3 grid(g.tiles_m * g.tiles_n), block(NTHR);
  const int group = config % 100, variant = config / 100 % 10;
  if (variant == 2 || variant == 3) {
    if (variant == 3) {
      if (group == 8) hipLaunchKernelGGL((gemm_w4d_kernel<AT, BT, ACC, 8, true>), grid, block, 0, stream(), g);
      else hipLaunchKernelGGL((gemm_w4d_kernel<AT, BT, ACC, 4, true>), grid, block, 0, stream(), g);
    } else {
      if (group == 8) hipLaunchKernelGGL((gemm_w4d_kernel<AT, BT, ACC, 8, false>), grid, block, 0, stream(), g);
      else hipLaunchKernelGGL((gemm_w4d_kernel<AT, BT, ACC, 4, false>), grid, block, 0, stream(), g);
    }
  } else if (variant == 1) {
    if (group == 8) hipLaunchKernelGGL((gemm_w4_kernel<AT, BT, ACC, 8, true>), grid, block, 0, stream(), g);
    else hipLaunchKernelGGL((gemm_w4_kernel<AT, BT, ACC, 4, true>), grid, block, 0, stream(), g);
  } else {
    if (group == 8) hipLaunchKernelGGL((gemm_w4_kernel<AT, BT, ACC, 8, false>), grid, block, 0, stream(), g);
    else hipLaunchKernelGGL((gemm_w4_kernel<AT, BT, ACC, 4, false>), grid, block, 0, stream(), g);
  }
}

}  // namespace

void gemm_w4_ex(const at::Tensor& a, const at::Tensor& b, at::Tensor& out, bool at_, bool bt_, bool accumulate,
                int64_t config) {
  LLMCTL_CHECK(a.dim() == 2 && b.dim() == 2 && out.dim() == 2, "gemm_w4_ex: 2-D operands");
  LLMCTL_CHECK(a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16 &&
                   out.scalar_type() == at::kBFloat16, "gemm_w4_ex: bf16 operands");
  LLMCTL_CHECK(a.is_cuda() && b.is_cuda() && out.is_cuda(), "gemm_w4_ex: GPU tensors");
  LLMCTL_CHECK(a.stride(1) == 1 && b.stride(1) == 1 && out.stride(1) == 1, "gemm_w4_ex: unit inner stride");
  const long M = at_ ? a.size(1) : a.size(0);
  const long K = at_ ? a.size(0) : a.size(1);
  const long N = bt_ ? b.size(1) : b.size(0);
  const long Kb = bt_ ? b.size(0) : b.size(1);
  LLMCTL_CHECK(K == Kb, "gemm_w4_ex: K mismatch");
  LLMCTL_CHECK(out.size(0) == M && out.size(1) == N, "gemm_w4_ex: out must be [M,N]");
  LLMCTL_CHECK(M % TM == 0 && N % TN == 0 && K % (2 * TK) == 0 && K > 0,
               "gemm_w4_ex: M,N multiples of 256, K of 128 (got ", M, "x", N, "x", K, ")");
  LLMCTL_CHECK(a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0 && out.stride(0) % 4 == 0 &&
                   (reinterpret_cast<uintptr_t>(a.data_ptr()) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(b.data_ptr()) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(out.data_ptr()) & 7) == 0,
               "gemm_w4_ex: 16-byte aligned operand rows");
  const long a_span = at_ ? K * a.stride(0) * 2 : (long)TM * a.stride(0) * 2;
  const long b_span = bt_ ? K * b.stride(0) * 2 : (long)TN * b.stride(0) * 2;
  LLMCTL_CHECK(a_span < (1L << 31) && b_span < (1L << 31), "gemm_w4_ex: operand too large for 32-bit offsets");
  const c10::DeviceGuard dg(a.device());
  W4Args g{reinterpret_cast<const unsigned short*>(a.data_ptr()), reinterpret_cast<const unsigned short*>(b.data_ptr()),
           reinterpret_cast<unsigned short*>(out.data_ptr()), a.stride(0), b.stride(0), out.stride(0),
           (int)M, (int)N, (int)K, (int)(M / TM), (int)(N / TN)};
  const int grp = (int)config;
  const int sel = (at_ ? 4 : 0) | (bt_ ? 2 : 0) | (accumulate ? 1 : 0);
  switch (sel) {
    case 0: launch<false, false, false>(g, grp); break;
    case 1: launch<false, false, true>(g, grp); break;
    case 2: launch<false, true, false>(g, grp); break;
    case 3: launch<false, true, true>(g, grp); break;
    case 4: launch<true, false, false>(g, grp); break;
    case 5: launch<true, false, true>(g, grp); break;
    case 6: launch<true, true, false>(g, grp); break;
    default: launch<true, true, true>(g, grp); break;
  }
}

TORCH_LIBRARY_IMPL(llmctl, CUDA, m) { m.impl("gemm_w4_ex", &gemm_w4_ex); }

}  // namespace llmctl
