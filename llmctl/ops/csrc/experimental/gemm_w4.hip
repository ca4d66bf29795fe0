// EXPERIMENT (not built: llmctl/ops/build.py compiles csrc/*.hip only).  Status: hipcc (ROCm 7.2)
// does not keep the 256 accumulators in AGPRs here — the main loop carries ~350 v_accvgpr_*
// moves per 128 MFMAs and a few spills (see the round-2 notes in README.md), so the design needs
// inline-asm MFMAs on named AGPRs before it can be measured.
//
// bf16 MFMA GEMM, 256x256 tile, ONE wave per SIMD (4 waves x 128x128 outputs), register-staged
// 64-deep K-tiles (gfx950).
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

__device__ __forceinline__ f32x4_t mfma16(bf16x8_t a, bf16x8_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
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

template <bool AT, bool BT, bool ACC, int GROUP>
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
  i32x4_t st[PIECES];  // register stage: half a K-tile (one operand) of this thread's pieces

  // one operand of K-tile t (clamped: past-the-end loads re-read the last tile) -> stage
  auto gload = [&](auto op_c, int t) {
    constexpr bool isA = decltype(op_c)::value == 0;
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
  // stage -> wbuf (operand OP) and the reload of that stage piece from K-tile t_load.
  auto part = [&](auto c_c, const unsigned char* rbuf, int rks, auto op_c, unsigned char* wbuf, int t_load) {
    constexpr int C = decltype(c_c)::value, N = 1 - C;
    constexpr bool isA = decltype(op_c)::value == 0;
    unsigned char* img = wbuf + (isA ? 0 : IMG);
    const int tc = t_load < KT ? t_load : KT - 1;
    const unsigned so0 = (unsigned)tc * (isA ? a_kstep : b_kstep);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i][j] = mfma16(fb[C][j], fa[C][i], acc[i][j]);
      fa[N][j] = frag<AT>(rbuf, am + 16 * j, rks, lane);
      fb[N][j] = frag<BT>(rbuf + IMG, bn + 16 * j, rks, lane);
      const unsigned lo = (j & 1) ? (isA ? alo1 : blo1) : (isA ? alo0 : blo0);
      *reinterpret_cast<i32x4_t*>(img + lo + 4096 * j) = st[j];
      const int so = __builtin_amdgcn_readfirstlane((int)(so0 + j * (isA ? aps : bps)));
      st[j] = __builtin_amdgcn_raw_buffer_load_b128(isA ? ra : rb, isA ? avo : bvo, so, 0);
      // keep this column's work together: 8 MFMA, the fragment reads, 1 ds_write, 1 load
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, (AT ? 2 : 1) + (BT ? 2 : 1), 0);
      __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    }
  };

  // prologue: K-tile 0 -> buffer 0, A(1) -> buffer 1, B(1) in the stage, frags (0, k0)
  gload(K_<0>{}, 0);
  swrite(K_<0>{}, smem);
  gload(K_<1>{}, 0);
  swrite(K_<1>{}, smem);
  gload(K_<0>{}, 1);
  swrite(K_<0>{}, smem + BUF);
  gload(K_<1>{}, 1);
  lds_sync();
  rfrags(K_<0>{}, smem, 0);

  // K-tile t in buf; nbuf holds K-tile t+1's A image (written in the previous part 2)
  auto ktile = [&](int t, unsigned char* buf, unsigned char* nbuf) {
    // part 1: MFMA(t, k0..31) | frags (t, k32..63) | B(t+1) stage -> nbuf | load A(t+2)
    part(K_<0>{}, buf, 1, K_<1>{}, nbuf, t + 2);
    lds_sync();  // K-tile t+1 complete and visible; every wave is done reading buf
    // part 2: MFMA(t, k32..63) | frags (t+1, k0..31) | A(t+2) stage -> buf | load B(t+2)
    part(K_<1>{}, nbuf, 0, K_<0>{}, buf, t + 2);
  };

  // one K-tile per iteration (buffers picked by parity at run time): a 2x-unrolled body gets
  // different accumulator registers in its two copies and hipcc then permutes all 256 AGPRs
  // with v_accvgpr_mov at every iteration
  for (int t = 0; t < KT; ++t) {
    unsigned char* buf = smem + (t & 1) * BUF;
    ktile(t, buf, smem + ((t + 1) & 1) * BUF);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the clamped tail loads

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

template <bool AT, bool BT, bool ACC>
void launch(const W4Args& g, int group) {
  const dim3 grid(g.tiles_m * g.tiles_n), block(NTHR);
  if (group == 8) hipLaunchKernelGGL((gemm_w4_kernel<AT, BT, ACC, 8>), grid, block, 0, stream(), g);
  else hipLaunchKernelGGL((gemm_w4_kernel<AT, BT, ACC, 4>), grid, block, 0, stream(), g);
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
