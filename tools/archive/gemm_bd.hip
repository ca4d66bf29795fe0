// "B direct" GEMM (gfx950, round 6 experiment): C[M, N] = A[M, K] B[N, K]^T, both operands
// K-contiguous (the forward projection x W^T; the data gradient dy (W^T)^T on the W^T copy).
//
// Why: the persistent gemm64 kernel stages BOTH operands through LDS by LDS-DMA, and its per-phase
// stamps put the loss in that per-CU LDS-DMA stream -- dropping either operand's DMA lifted it from
// ~1.4 to 1.8-1.96 PF (profiles/gemm_probe_r4.txt).  Here only A goes through LDS; the four waves
// stand side by side on 64-column slices of the 256 x 256 tile (each wave: all 256 rows x its 64
// columns, 16 x 4 MFMA 16x16x32 blocks, 256 AGPR accumulators), so every B row is loaded by exactly
// one wave, straight into registers, in the MFMA operand layout:
//   * MFMA step s of lane group g covers k = 32 s + 8 g + [0, 8) of each 64-deep K-tile: one B load
//     instruction reads 64 contiguous bytes of each of its 16 weight rows, the pair a full 128-B line;
//   * A: 256 rows x 64 k per K-tile = 32 KB, source-swizzled row image (16-B chunk c of row r at
//     c ^ ((r >> 1) & 7): conflict-free ds_read_b128 for 16 rows at one chunk), 4 stages;
//   * one barrier per K-tile (the DMA of tile t+3 is issued after tile t's barrier, into the stage
//     tile t-1 used); B fragments of tiles t..t+3 live in registers (4 slots x 32 VGPRs);
//   * vmcnt: per K-tile each thread issues 8 DMA pieces then 8 B loads (asm, manual counts): at
//     tile t, 32 younger ops (tiles t+1, t+2) may stay in flight.
// One-shot grid (one tile per workgroup, XCD-aware order): this is the core-loop experiment.
#include <utility>

#include "attn_common.h"

namespace llmctl {
namespace {

using namespace attn;
using f32x4_t = __attribute__((ext_vector_type(4))) float;
using i32x4_t = __attribute__((ext_vector_type(4))) int;

constexpr int BM = 256, BN = 256, BK = 64, STG = 4;
constexpr int ASTAGE = BM * BK * 2;  // 32 KB

struct BdArgs {
  const unsigned short* a;
  const unsigned short* b;
  unsigned short* c;
  int M, N, K;
  long lda, ldb, ldc;
  int tiles_m, tiles_n, group;
};

__device__ __forceinline__ i32x4_t rsrc_of(const void* base) {
  const unsigned long p = (unsigned long)base;
  i32x4_t r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(p & 0xffffffffu));
  r[1] = __builtin_amdgcn_readfirstlane((int)((p >> 32) & 0xffff));
  r[2] = -1;
  r[3] = 0x00020000;
  return r;
}

// LDS-DMA piece: 64 lanes x 16 B -> LDS [lds_byte, +1024), lane-linear
__device__ __forceinline__ void dma16(i32x4_t rsrc, unsigned voff, unsigned soff, unsigned lds_byte) {
  asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(voff), "s"(rsrc),
               "s"(soff), "s"(lds_byte)
               : "memory");
}

// B fragment pair of one n-block: 32 contiguous bytes (k-steps 0 and 1) -- asm, so that the
// compiler's vmcnt bookkeeping (blind to the asm DMA) does not drain the stream; the waits are ours
__device__ __forceinline__ void bload(bf16x8_t& lo, bf16x8_t& hi, i32x4_t rsrc, unsigned voff, unsigned soff) {
  asm volatile("buffer_load_dwordx4 %0, %2, %3, %4 offen\n\t"
               "buffer_load_dwordx4 %1, %2, %3, %4 offen offset:64"
               : "=&v"(lo), "=&v"(hi)
               : "v"(voff), "s"(rsrc), "s"(soff)
               : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// c0 += B0 x A, c1 += B1 x A (swapped product: lane holds C[m = l & 15][n = 4 (l >> 4) + r])
__device__ __forceinline__ void mfma_pair(f32x4_t& c0, f32x4_t& c1, const bf16x8_t& a, const bf16x8_t& b0,
                                          const bf16x8_t& b1) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %3, %2, %0\n\t"
               "v_mfma_f32_16x16x32_bf16 %1, %4, %2, %1"
               : "+a"(c0), "+a"(c1)
               : "v"(a), "v"(b0), "v"(b1)
               : "memory");
}
__device__ __forceinline__ void mfma_pair_z(f32x4_t& c0, f32x4_t& c1, const bf16x8_t& a, const bf16x8_t& b0,
                                            const bf16x8_t& b1) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %3, %2, 0\n\t"
               "v_mfma_f32_16x16x32_bf16 %1, %4, %2, 0"
               : "=a"(c0), "=a"(c1)
               : "v"(a), "v"(b0), "v"(b1)
               : "memory");
}

__device__ __forceinline__ int swr(int row) { return (row >> 1) & 7; }

template <typename F, int... Q>
__device__ __forceinline__ void unroll_seq(F&& f, std::integer_sequence<int, Q...>) {
  (f(std::integral_constant<int, Q>{}), ...);
}

// EXP (timing ablations, results garbage): 1 = no B loads in the loop, 2 = no A DMA in the loop, 3 = no barrier;
// 4 = (correct) all of a K-tile's loads issued right after the barrier instead of one per MFMA gap
template <int EXP>
__global__ __launch_bounds__(256, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm_bd_kernel(BdArgs args) {
  __shared__ __attribute__((aligned(1024))) unsigned char smem[STG * ASTAGE];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware order (consecutive ids of one XCD get consecutive tiles), then GROUP-row swizzle
  int tm, tn;
  {
    const int bid = blockIdx.x, nwg = args.tiles_m * args.tiles_n;
    const int q = nwg / 8, rem = nwg % 8, x = bid % 8;
    const int wg = (x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q) + bid / 8;
    const int per_group = args.group * args.tiles_n;
    const int grp = wg / per_group;
    const int gsz = min(args.group, args.tiles_m - grp * args.group);
    const int inner = wg - grp * per_group;
    tm = grp * args.group + inner % gsz;
    tn = inner / gsz;
  }
  const long lda = args.lda, ldb = args.ldb;
  const i32x4_t rA = rsrc_of(args.a + (long)tm * BM * lda);
  const i32x4_t rB = rsrc_of(args.b + ((long)tn * BN + 64 * w) * ldb);
  unsigned voA[8], voB[4];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int p = w * 8 + j;  // this wave's DMA pieces: image rows 8p .. 8p + 7
    const int row = 8 * p + (lane >> 3), pc = lane & 7;
    voA[j] = (unsigned)(((long)row * lda + ((pc ^ swr(row)) << 3)) * 2);
  }
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) voB[nb] = (unsigned)(((long)(16 * nb + (lane & 15)) * ldb + 8 * (lane >> 4)) * 2);
  const unsigned lds0 = lds_addr(smem);
  const int KT = args.K / BK;

  bf16x8_t bq[4][4][2];  // [slot = K-tile & 3][n-block][k-step]
  // vector-memory op o (0..15) of K-tile t's stream: o < 8 the A DMA piece o, else the B fragment pair
  // of n-block o - 8 -- placed one per MFMA gap by the K loop (EXP 4: all 16 right after the barrier)
  auto issue_op = [&](int t, auto slot_c, auto o_c) __attribute__((always_inline)) {
    constexpr int SL = decltype(slot_c)::value;
    constexpr int O = decltype(o_c)::value;
    const int tc = t < KT ? t : KT - 1;  // past the end: re-load the last tile (nobody reads it)
    const unsigned so = (unsigned)tc * BK * 2;
    if constexpr (O < 8) {
      if (EXP != 2 || t < 3) dma16(rA, voA[O], so, lds0 + (unsigned)(t % STG) * ASTAGE + (w * 8 + O) * 1024);
    } else {
      if (EXP != 1 || t < 4) bload(bq[SL][O - 8][0], bq[SL][O - 8][1], rB, voB[O - 8], so);
    }
  };
  auto issue = [&](int t, auto slot_c) __attribute__((always_inline)) {
    issue_op(t, slot_c, std::integral_constant<int, 0>{});
    issue_op(t, slot_c, std::integral_constant<int, 1>{});
    issue_op(t, slot_c, std::integral_constant<int, 2>{});
    issue_op(t, slot_c, std::integral_constant<int, 3>{});
    issue_op(t, slot_c, std::integral_constant<int, 4>{});
    issue_op(t, slot_c, std::integral_constant<int, 5>{});
    issue_op(t, slot_c, std::integral_constant<int, 6>{});
    issue_op(t, slot_c, std::integral_constant<int, 7>{});
    issue_op(t, slot_c, std::integral_constant<int, 8>{});
    issue_op(t, slot_c, std::integral_constant<int, 9>{});
    issue_op(t, slot_c, std::integral_constant<int, 10>{});
    issue_op(t, slot_c, std::integral_constant<int, 11>{});
  };

  f32x4_t acc[16][4];
  // fragment of row block rb, k-step s from stage SL: lane (i = l & 15, g = l >> 4) reads row 16 rb + i at
  // chunk 4 s + g; the swizzle (row >> 1) & 7 = (i >> 1) & 7 does not depend on rb, so the per-lane
  // part is two offsets (s = 0, 1) and stage / row block are immediates
  const int i16 = lane & 15;
  const unsigned abase[2] = {(unsigned)(i16 * 128 + (((lane >> 4) ^ swr(i16)) << 4)),
                             (unsigned)(i16 * 128 + (((4 + (lane >> 4)) ^ swr(i16)) << 4))};
  auto afrag = [&](auto st_c, int rb, int s) __attribute__((always_inline)) {
    constexpr int ST = decltype(st_c)::value;
    return *reinterpret_cast<const bf16x8_t*>(smem + ST * ASTAGE + rb * 2048 + abase[s]);
  };
  auto ktile = [&](int t, auto slot_c, auto zero_c) __attribute__((always_inline)) {
    constexpr int SL = decltype(slot_c)::value;
    constexpr bool Z = decltype(zero_c)::value;
    wait_vm<(EXP == 1 || EXP == 2) ? 16 : 32>();  // tile t's A pieces and B fragments (t+1, t+2 stay in flight)
    if constexpr (EXP != 3) __builtin_amdgcn_s_barrier();
    constexpr int NS = (SL + 3) & 3;
    if constexpr (EXP == 4) issue(t + 3, std::integral_constant<int, NS>{});
    bf16x8_t af[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) af[q] = afrag(slot_c, q & 15, q >> 4);
    auto body = [&](auto q_c) __attribute__((always_inline)) {
      constexpr int q = decltype(q_c)::value;
      constexpr int rb = q & 15, s = q >> 4;
      if (Z && s == 0) {
        mfma_pair_z(acc[rb][0], acc[rb][1], af[q & 7], bq[SL][0][s], bq[SL][1][s]);
        mfma_pair_z(acc[rb][2], acc[rb][3], af[q & 7], bq[SL][2][s], bq[SL][3][s]);
      } else {
        mfma_pair(acc[rb][0], acc[rb][1], af[q & 7], bq[SL][0][s], bq[SL][1][s]);
        mfma_pair(acc[rb][2], acc[rb][3], af[q & 7], bq[SL][2][s], bq[SL][3][s]);
      }
      if constexpr (q + 8 < 32) af[q & 7] = afrag(slot_c, (q + 8) & 15, (q + 8) >> 4);
      // the next K-tile's 12 vector-memory ops, one per MFMA gap (2 pairs) from the second statement
      if constexpr (EXP != 4 && q >= 1 && q < 25 && (q - 1) % 2 == 0)
        issue_op(t + 3, std::integral_constant<int, NS>{}, std::integral_constant<int, (q - 1) / 2>{});
    };
    unroll_seq(body, std::make_integer_sequence<int, 32>{});
    // every wave's reads of this stage are done before the next barrier (WAR: tile t+4's DMA)
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  };

  issue(0, std::integral_constant<int, 0>{});
  issue(1, std::integral_constant<int, 1>{});
  issue(2, std::integral_constant<int, 2>{});
  ktile(0, std::integral_constant<int, 0>{}, std::true_type{});
  ktile(1, std::integral_constant<int, 1>{}, std::false_type{});
  ktile(2, std::integral_constant<int, 2>{}, std::false_type{});
  ktile(3, std::integral_constant<int, 3>{}, std::false_type{});
  for (int t = 4; t < KT; t += 4) {
    ktile(t, std::integral_constant<int, 0>{}, std::false_type{});
    ktile(t + 1, std::integral_constant<int, 1>{}, std::false_type{});
    ktile(t + 2, std::integral_constant<int, 2>{}, std::false_type{});
    ktile(t + 3, std::integral_constant<int, 3>{}, std::false_type{});
  }
  wait_vm<0>();  // the past-the-end re-loads
  // last MFMAs -> accumulator reads by the stores below: wait states
  asm volatile("s_nop 7\n\ts_nop 7"
               : "+a"(acc[15][0]), "+a"(acc[15][1]), "+a"(acc[15][2]), "+a"(acc[15][3]), "+a"(acc[14][0]),
                 "+a"(acc[14][1]), "+a"(acc[14][2]), "+a"(acc[14][3]));
  // bf16 stores, 16 B per lane: v_permlane16_swap pairs n-blocks (0, 1) and (2, 3) so a lane holds 8
  // consecutive columns 32 jp + 16 (g & 1) + 8 (g >> 1) + [0, 8) of row m
  const int g = lane >> 4;
  unsigned short* Cb = args.c + ((long)tm * BM + (lane & 15)) * args.ldc + (long)tn * BN + 64 * w + 16 * (g & 1) +
                       8 * (g >> 1);
#pragma unroll
  for (int rb = 0; rb < 16; ++rb) {
#pragma unroll
    for (int jp = 0; jp < 2; ++jp) {
      const int j = 2 * jp;
      const unsigned x0 = (unsigned)f2bf(acc[rb][j][0]) | ((unsigned)f2bf(acc[rb][j][1]) << 16);
      const unsigned x1 = (unsigned)f2bf(acc[rb][j][2]) | ((unsigned)f2bf(acc[rb][j][3]) << 16);
      const unsigned y0 = (unsigned)f2bf(acc[rb][j + 1][0]) | ((unsigned)f2bf(acc[rb][j + 1][1]) << 16);
      const unsigned y1 = (unsigned)f2bf(acc[rb][j + 1][2]) | ((unsigned)f2bf(acc[rb][j + 1][3]) << 16);
      const auto r0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
      const auto r1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
      *reinterpret_cast<uint4*>(Cb + (long)(16 * rb) * args.ldc + 32 * jp) = make_uint4(r0[0], r1[0], r0[1], r1[1]);
    }
  }
}

}  // namespace

// C [M, N] = A [M, K] . B [N, K]^T (bf16, both K-contiguous): the B-direct experiment kernel.
// M, N multiples of 256, K a multiple of 256 (>= 256); row strides = K (A, B) and N (C).
at::Tensor gemm_bd(const at::Tensor& a, const at::Tensor& b, int64_t group) {
  LLMCTL_CHECK(a.dim() == 2 && b.dim() == 2 && a.is_contiguous() && b.is_contiguous() && a.is_cuda() && b.is_cuda() &&
                   a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16,
               "gemm_bd: 2-D contiguous bf16 GPU operands");
  const int M = a.size(0), K = a.size(1), N = b.size(0);
  LLMCTL_CHECK(b.size(1) == K && M % BM == 0 && N % BN == 0 && K % (4 * BK) == 0 && K >= 4 * BK,
               "gemm_bd: M, N multiples of 256, K a multiple of 256");
  LLMCTL_CHECK((long)BM * K * 2 < (1L << 31), "gemm_bd: a tile's operand bytes must fit the 32-bit buffer offsets");
  const c10::DeviceGuard guard(a.device());
  auto c = at::empty({M, N}, a.options());
  BdArgs args{bf_ptr(a), bf_ptr(b), bf_mut(c), M, N, K, K, K, N, M / BM, N / BN, (int)std::max<int64_t>(1, group)};
  const dim3 grid(args.tiles_m * args.tiles_n);
  switch (knob("bd_exp", 0)) {
    case 1: hipLaunchKernelGGL(gemm_bd_kernel<1>, grid, dim3(256), 0, stream(), args); break;
    case 2: hipLaunchKernelGGL(gemm_bd_kernel<2>, grid, dim3(256), 0, stream(), args); break;
    case 3: hipLaunchKernelGGL(gemm_bd_kernel<3>, grid, dim3(256), 0, stream(), args); break;
    case 4: hipLaunchKernelGGL(gemm_bd_kernel<4>, grid, dim3(256), 0, stream(), args); break;
    default: hipLaunchKernelGGL(gemm_bd_kernel<0>, grid, dim3(256), 0, stream(), args);
  }
  return c;
}

TORCH_LIBRARY_IMPL(llmctl, CUDA, m) { m.impl("gemm_bd", &gemm_bd); }

}  // namespace llmctl
