// Pointwise (1x1) convolution as a persistent, LDS-DMA-pipelined MFMA GEMM (gfx950).
//
//   OUT[m][n] = sum_k A[m][k] * B[n][k]        A = NHWC activation rows (m = output pixel; a
//                                              stride-2 1x1 conv gathers rows (n, 2p, 2q)),
//                                              B = weights [Cout][Cin], k = input channel
//
// ResNet-50's bottleneck 1x1s (`pytorch_model.py:44-49`, 2/3 of its forward FLOPs) and
// MobileNetV2's expand / project convs are plain GEMMs in NHWC, scored at B = 1280 / 320
// (`pytorch_collab.py:95-103`): M = 62k..4M rows, K and N = 64..2048.  Most of these shapes sit
// near the HBM/MFMA balance point, so the design goal is to stream A from HBM ONCE at full rate
// while the matrix cores stay busy:
//
//   * persistent: one 512-thread block per CU walks a CONTIGUOUS range of 256-row output tiles
//     (N-tiles of one M panel back to back, so the panel's re-reads are L2 hits) as one
//     continuous stream of K-steps -- the next tile's first operand tiles are in flight while
//     the current tile finishes and while its epilogue stores drain;
//   * operands go HBM -> LDS by buffer LDS-DMA (`buffer_load_dwordx4 ... lds`, 1 KB per wave
//     instruction) into an S-slot ring of (256 + BN) x 32 bf16 K-steps; waits are counted
//     `s_waitcnt vmcnt(N)` + raw `s_barrier`, so S - 2 steps stay in flight across every
//     barrier and nothing drains the ring (no compiler-visible global load inside the loop);
//   * padding (rows past M, channels past N, K not a multiple of 32) costs nothing: those
//     lanes' DMA offsets point past the buffer resource's range, which lands zeros; stores to
//     such offsets are dropped by the same range check;
//   * 8 waves (two per SIMD), 16x16x32 bf16 MFMA with weights as the MFMA "A" operand, so each
//     lane's accumulator holds 4 consecutive channels of one pixel (8 contiguous NHWC bytes):
//     the epilogue stores straight from registers and reduces the ghost-BN statistics (sum,
//     sum of squares per channel and 32-image group) with DPP row sums;
//   * step s + 1's fragments are read from LDS while step s's MFMAs issue
//     (`sched_group_barrier` interleave);
//   * LDS rows are 64 B (one K-step); chunk c of row r lives at chunk c ^ ((r >> 1) & 3), which
//     makes every ds_read_b128 fragment read conflict-free for the four 16-lane groups of
//     gfx950 (checked exhaustively on the host, `bench/lds_swizzle_check.py`); the DMA side
//     applies the inverse permutation on the SOURCE address (the LDS image is lane-linear).
#include <stdlib.h>

#include "common.h"
#include "igemm.h"

namespace {

constexpr int PG_BM = 256;        // output rows per tile
constexpr int PG_BK = 32;         // K per step (one 16x16x32 MFMA k-block)
constexpr int PG_NW = 8;          // waves per block
constexpr int PG_NT = 64 * PG_NW;
constexpr unsigned PG_OOB = 0xFFFFFF00u;   // byte offset past every tensor: zeros / dropped

MA_DEV unsigned pg_lds_addr(const void* p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) char*)p;
}

MA_DEV __amdgpu_buffer_rsrc_t pg_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, bytes, 0x00020000);
}

// 16 bytes per lane, buffer -> LDS; lane l lands at the wave-uniform LDS byte address + 16 l.
// Inline asm on purpose: hipcc models LDS-DMA as an LDS event and would then answer every
// fragment read with lgkmcnt(0) / drain the ring; completion is tracked by our own vmcnt waits.
MA_DEV void pg_dma16(__amdgpu_buffer_rsrc_t r, unsigned off, unsigned lds) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
               ::"v"(off), "s"(r), "s"(lds) : "memory");
}

template <int N>
MA_DEV void pg_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// barrier without __syncthreads' release fence (its vmcnt(0) would drain the DMA ring)
MA_DEV void pg_bar() { asm volatile("s_barrier" ::: "memory"); }

MA_DEV float pg_row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  return v;
}

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// Output-channel order of the weight tile in LDS: within every 32 rows, LDS row
// h * 16 + 4 q + j (fragment half h, lane group q, accumulator element j) holds channel
// 8 q + 4 h + j, so a lane's accumulators of the fragment pair (2t, 2t + 1) are 8 CONSECUTIVE
// channels of one pixel: the epilogue leaves as 16-byte stores (16 pixels x 64 contiguous bytes
// per wave instruction instead of 16 x 32)
MA_DEV int pg_perm(int r) {
  const int r5 = r & 31;
  return (r & ~31) | (((r5 >> 2) & 3) << 3) | ((r5 >> 4) << 2) | (r5 & 3);
}

// wait until a step's DMA pieces have landed: `newer` = whole steps (P pieces each) this wave
// issued after it (0 .. S-2; wave-uniform, so the branches are scalar).  VMEM ops issued after
// those (epilogue stores, stat atomics) are not counted: the wait then also covers some of
// them -- longer, never too short.
template <int P>
MA_DEV void pg_wait_steps(int newer) {
  switch (newer) {
    case 0: pg_wait<0>(); break;
    case 1: pg_wait<P>(); break;
    case 2: pg_wait<2 * P>(); break;
    case 3: pg_wait<3 * P>(); break;
    default: pg_wait<4 * P>(); break;
  }
}

template <int BN, int WM, int S, bool STATS, bool GATHER, int MODE>
__global__ __launch_bounds__(PG_NT, 1) void pgemm_kernel(PgemmArgs g, PgemmPro pro) {
  constexpr int BM = PG_BM, WN = PG_NW / WM;
  constexpr int TM = BM / (16 * WM), TN = BN / (16 * WN);
  constexpr int PA = BM / 16 / PG_NW;                     // A pieces per wave per step
  constexpr int PB = BN >= 128 ? BN / 16 / PG_NW : 1;     // B pieces (BN = 64: waves 4-7 dump)
  // MODE > 0: + one coefficient piece per wave (its own copy: read after its own vmcnt, no
  // barrier), MODE 2: + the residual tile's pieces
  constexpr int PC = MODE > 0 ? 1 : 0, PR = MODE == 2 ? PA : 0;
  constexpr int P = PA + PB + PC + PR;
  constexpr int SA = BM * 64, SB = BN * 64, SC = PC * PG_NW * 1024, SR = PR ? SA : 0;
  constexpr int SLOT = SA + SB + SC + SR;
  static_assert(!(GATHER && MODE), "input prologue: stride-1 convs only");
  static_assert(TM >= 1 && TN >= 1 && PA >= 1, "tile shape");
  static_assert(S >= 3 && S <= 6, "ring depth (pg_wait_steps covers newer <= 4)");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const int wm = w / WN, wn = w % WN;
  const int ntn = (g.N + BN - 1) / BN;
  const int mtiles = (g.M + BM - 1) / BM;
  const int ntiles = mtiles * ntn;
  // contiguous tile range of this block (N-tiles of one M panel consecutive)
  const int G = gridDim.x, b = blockIdx.x;
  const int t_begin = (int)((long long)ntiles * b / G), t_end = (int)((long long)ntiles * (b + 1) / G);
  if (t_begin >= t_end) return;
  const int KT = (g.K + PG_BK - 1) / PG_BK;               // K-steps per tile
  const int NS = (t_end - t_begin) * KT;                  // steps of this block

  const auto rs_a = pg_rsrc(g.a, g.a_bytes);
  const auto rs_b = pg_rsrc(g.b, g.b_bytes);
  const auto rs_o = pg_rsrc(g.out, g.out_bytes);
  const unsigned s_ring = pg_lds_addr(smem);
  const unsigned s_dump = s_ring + S * SLOT + wu * 1024;
  (void)SR;

  // ---- DMA lane roles: piece row (lane >> 2), physical chunk (lane & 3), logical chunk lc
  const int prow = lane >> 2;
  const int lc = (lane & 3) ^ ((prow >> 1) & 3);
  const bool kfull = (g.K & 31) == 0;
  const int K8 = g.K >> 3;                                // 16-byte chunks per row
  unsigned aoff[PA], boff[PB];                            // per tile: row byte offset + lc
  unsigned coff = PG_OOB;                                 // MODE > 0: this lane's coef source
  const auto rs_c = pg_rsrc(pro.coef, pro.coef_bytes);
  const auto rs_r = pg_rsrc(pro.res, pro.res_bytes);
  const auto rs_k = pg_rsrc(pro.keep, pro.keep_bytes);
  auto set_tile = [&](int t) {
    const int mt = t / ntn, nt = t - mt * ntn;
    if constexpr (MODE > 0) {
      // lanes 0-7 scale, 8-15 shift of the tile's first group; 16-31 the same for the next
      // group (a tile straddles at most one group edge); channel offset added per step
      const int gq = (mt * BM) / pro.group_rows + ((lane >> 4) & 1);
      const int which = (lane >> 3) & 1;
      coff = (lane < 32 && gq < pro.G) ? (unsigned)(((gq * 2 + which) * g.K + 4 * (lane & 7)) * 4)
                                       : PG_OOB;
    }
#pragma unroll
    for (int j = 0; j < PA; ++j) {
      const int m = mt * BM + 16 * (wu + PG_NW * j) + prow;
      int src = m;
      if constexpr (GATHER) {
        const int pq = g.P * g.Q;
        const int n = m / pq, rem = m - n * pq;
        const int p = rem / g.Q, q = rem - p * g.Q;
        src = (n * g.H + p * g.stride) * g.W + q * g.stride;
      }
      aoff[j] = m < g.M ? (unsigned)(((long long)src * g.K + lc * 8) * 2) : PG_OOB;
    }
#pragma unroll
    for (int j = 0; j < PB; ++j) {
      const int nr = 16 * (wu + PG_NW * j) + prow;
      const int n = nt * BN + pg_perm(nr);
      boff[j] = (n < g.N && nr < BN) ? (unsigned)((n * g.K + lc * 8) * 2) : PG_OOB;
    }
  };
  // DMA piece q (0 .. P-1) of K-step kt into ring slot `slot`: A pieces first, then B
  auto issue_piece = [&](int q, int kt, int slot) {
    const unsigned kb = (unsigned)(kt * 64);
    const bool kok = kfull || kt * 4 + lc < K8;
    const unsigned sa = s_ring + slot * SLOT, sb = sa + SA;
    if (q < PA) {
      pg_dma16(rs_a, kok ? aoff[q] + kb : PG_OOB, sa + 16 * (wu + PG_NW * q) * 64);
    } else if (q < PA + PB) {
      const int j = q - PA;
      const bool real = 16 * (wu + PG_NW * j) < BN;
      pg_dma16(rs_b, kok ? boff[j] + kb : PG_OOB, real ? sb + 16 * (wu + PG_NW * j) * 64 : s_dump);
    } else if (q < PA + PB + PC) {
      // 32 channels of this step: 128 B of scale / shift per group (channels past K: zeros)
      const bool cok = kt * 32 + 4 * (lane & 7) < g.K;
      pg_dma16(rs_c, coff != PG_OOB && cok ? coff + (unsigned)(kt * 128) : PG_OOB,
               sa + SA + SB + wu * 1024);
    } else {
      const int j = q - PA - PB - PC;
      pg_dma16(rs_r, kok ? aoff[j] + kb : PG_OOB, sa + SA + SB + SC + 16 * (wu + PG_NW * j) * 64);
    }
  };

  // ---- MODE > 0: normalise this thread's own landed A chunks of a step in place (after its
  // own vmcnt wait, before the barrier that publishes the step): a = act(y * scale + shift
  // [+ res]); N-tile-0 tiles also write the activation to ``keep``
  float clo = 0.f, chi = 0.f;
  if constexpr (MODE > 0) {
    clo = pro.act == 0 ? __builtin_nanf("") : 0.f;          // NaN bounds: identity, keeps NaN
    chi = pro.act == 2 ? 6.f : (pro.act == 0 ? __builtin_nanf("") : __builtin_huge_valf());
  }
  auto transform = [&](int tt, int ktt, int sl) {
    if constexpr (MODE > 0) {
      const int mt = tt / ntn, nt = tt - mt * ntn;
      const int m0 = mt * BM;
      const int bnd = (m0 / pro.group_rows + 1) * pro.group_rows;
      char* sa = smem + sl * SLOT;
      const char* cw = sa + SA + SB + wu * 1024;
#pragma unroll
      for (int j = 0; j < PA; ++j) {
        const int row = m0 + 16 * (wu + PG_NW * j) + prow;
        const int gs = row >= bnd ? 256 : 0;
        const f32x4 c0 = *(const f32x4*)(cw + gs + lc * 32), c1 = *(const f32x4*)(cw + gs + lc * 32 + 16);
        const f32x4 h0 = *(const f32x4*)(cw + gs + 128 + lc * 32),
                    h1 = *(const f32x4*)(cw + gs + 128 + lc * 32 + 16);
        u32x4* ap = (u32x4*)(sa + 16 * (wu + PG_NW * j) * 64 + lane * 16);
        const bf16x8 y = __builtin_bit_cast(bf16x8, *ap);
        bf16x8 r8;
        if constexpr (MODE == 2)
          r8 = __builtin_bit_cast(bf16x8, *(const u32x4*)(sa + SA + SB + SC + 16 * (wu + PG_NW * j) * 64 + lane * 16));
        bf16x8 o;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float v = bf2f(y[k]) * (k < 4 ? c0[k] : c1[k - 4]) + (k < 4 ? h0[k] : h1[k - 4]);
          if constexpr (MODE == 2) v += bf2f(r8[k]);
          o[k] = f2bf(fminf(fmaxf(v, clo), chi));
        }
        const u32x4 ov = __builtin_bit_cast(u32x4, o);
        *ap = ov;
        if (pro.keep != nullptr && nt == 0) {
          const bool ok = row < g.M && (kfull || ktt * 4 + lc < K8);
          const unsigned ko = ok ? (unsigned)(((long long)row * g.K + ktt * 32 + lc * 8) * 2) : PG_OOB;
          __builtin_amdgcn_raw_buffer_store_b128(ov, rs_k, ko, 0, 0);
        }
      }
    }
  };

  // ---- fragment read offsets (lane part constant: row & 15 = lane & 15)
  const int fl = (lane & 15) * 64 + 16 * ((lane >> 4) ^ ((lane >> 1) & 3));
  auto read_frags = [&](bf16x8 (&fa)[TM], bf16x8 (&fb)[TN], int slot) {
    const char* sa = smem + slot * SLOT;
    const char* sb = sa + SA;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
      fa[tm] = *(const bf16x8*)(sa + (wm * (BM / WM) + tm * 16) * 64 + fl);
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
      fb[tn] = *(const bf16x8*)(sb + (wn * (BN / WN) + tn * 16) * 64 + fl);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- ghost-BN statistics.  Per-lane partial sums (over this lane's pixel rows) are reduced
  // over the 16 pixel lanes by DPP, over the WM wave rows through LDS, and land as ONE atomic
  // pair per (channel, flush): the stat addresses are shared by every block, so per-wave atomics
  // serialised on them (measured: 8 wave rows x 15680 tiles on 5120 addresses dominated the
  // K = 64 convs).  With a single N-tile the block keeps RUNNING sums across its consecutive
  // tiles and flushes only when the statistics group changes (contiguous tile ranges: a few
  // flushes per block).
  float* red = (float*)(smem + S * SLOT + PG_NW * 1024);   // [WM][2][BN]
  const bool run = STATS && ntn == 1;
  float rs[TN][4], rss[TN][4];
#pragma unroll
  for (int tn = 0; tn < TN; ++tn)
#pragma unroll
    for (int j = 0; j < 4; ++j) rs[tn][j] = rss[tn][j] = 0.f;
  int rgrp = -1;
  auto flush = [&](int grp, int n0) {
    // rs / rss: per-lane partials of group grp, columns n0 + (this wave's) -> stats, then zero
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        rs[tn][j] = pg_row16_sum(rs[tn][j]);
        rss[tn][j] = pg_row16_sum(rss[tn][j]);
      }
      if ((lane & 15) == 0) {
        // (pg_perm: fragment tn = 2 t + h holds channels 32 t + 8 q + 4 h + j)
        const int cl = wn * (BN / WN) + (tn >> 1) * 32 + 8 * (lane >> 4) + 4 * (tn & 1);
        *(f32x4*)(red + (wm * 2) * BN + cl) = f32x4{rs[tn][0], rs[tn][1], rs[tn][2], rs[tn][3]};
        *(f32x4*)(red + (wm * 2 + 1) * BN + cl) = f32x4{rss[tn][0], rss[tn][1], rss[tn][2], rss[tn][3]};
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) rs[tn][j] = rss[tn][j] = 0.f;
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (tid < BN && n0 + tid < g.N) {
      float a = 0.f, c = 0.f;
#pragma unroll
      for (int q = 0; q < WM; ++q) {
        a += red[(q * 2) * BN + tid];
        c += red[(q * 2 + 1) * BN + tid];
      }
      float* dst = MA_SPREAD(g.stats + (size_t)grp * 2 * g.stats_ld + n0 + tid);
      atomicAdd(dst, a);
      atomicAdd(dst + g.stats_ld, c);
    }
    // the red area is rewritten no earlier than the next flush: a second flush in the same
    // epilogue (straddling tile) waits for these reads
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  };

  // ---- epilogue of one tile: bf16 round, 16-byte stores from the registers (a fragment pair's
  // 8 consecutive channels per lane, pg_perm), statistics
  static_assert(TN % 2 == 0, "fragment pairs");
  auto epilogue = [&](int t) {
    const int mt = t / ntn, nt = t - mt * ntn;
    const int m0 = mt * BM, n0 = nt * BN;
    const int rbase = m0 + wm * (BM / WM) + (lane & 15);
    const int cbase = n0 + wn * (BN / WN) + 8 * (lane >> 4);
    int g0 = 0, bnd = 0x7fffffff;
    bool straddle = false;
    if constexpr (STATS) {
      g0 = m0 / g.group_rows;
      bnd = (g0 + 1) * g.group_rows;
      straddle = bnd < m0 + BM && bnd < g.M;
      if (run && rgrp != g0) {
        if (rgrp >= 0) flush(rgrp, n0);
        rgrp = g0;
      }
    }
    // rows < bnd of this tile (all rows unless it straddles a group edge)
#pragma unroll
    for (int tp = 0; tp < TN / 2; ++tp) {
      const int col = cbase + tp * 32;
      const bool cok = col < g.N;                 // (N % 8 == 0: 8 channels whole or out)
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const int row = rbase + tm * 16;
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          o[j] = f2bf(acc[tm][2 * tp][j]);
          o[4 + j] = f2bf(acc[tm][2 * tp + 1][j]);
        }
        const bool ok = row < g.M && cok;
        const unsigned voff = ok ? (unsigned)(((long long)row * g.ldo + col) * 2) : PG_OOB;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rs_o, voff, 0, 0);
        if constexpr (STATS) {
          const float mk = row < g.M && row < bnd ? 1.f : 0.f;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float f = bf2f(o[j]) * mk, f2 = bf2f(o[4 + j]) * mk;
            rs[2 * tp][j] += f;
            rss[2 * tp][j] += f * f;
            rs[2 * tp + 1][j] += f2;
            rss[2 * tp + 1][j] += f2 * f2;
          }
        }
      }
    }
    if constexpr (STATS) {
      if (straddle || !run) flush(g0, n0);
      if (straddle) {
        // rows >= bnd: the next group (a tile straddles at most one edge: groups >= BM rows)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
#pragma unroll
          for (int tm = 0; tm < TM; ++tm) {
            const int row = rbase + tm * 16;
            const float mk = row < g.M && row >= bnd ? 1.f : 0.f;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float f = bf2f(f2bf(acc[tm][tn][j])) * mk;
              rs[tn][j] += f;
              rss[tn][j] += f * f;
            }
          }
        if (run) rgrp = g0 + 1;
        else flush(g0 + 1, n0);
      }
    }
  };

  // ---- prologue: steps 0 .. S-2 in flight, step 0's fragments in registers
  int t_issue = t_begin, kt_issue = 0;                    // next step to issue
  set_tile(t_issue);
  auto advance_issue = [&]() {
    if (++kt_issue == KT) {
      kt_issue = 0;
      if (++t_issue < t_end) set_tile(t_issue);
    }
  };
  const int pro_n = NS < S - 1 ? NS : S - 1;
  for (int i = 0; i < pro_n; ++i) {
#pragma unroll
    for (int q = 0; q < P; ++q) issue_piece(q, kt_issue, i);
    advance_issue();
  }
  pg_wait_steps<P>(pro_n - 1);                            // step 0 landed
  int t_x = t_begin, kt_x = 0;                            // step the next transform handles
  transform(t_x, kt_x, 0);
  auto advance_x = [&]() {
    if (++kt_x == KT) kt_x = 0, ++t_x;
  };
  advance_x();
  if constexpr (MODE > 0) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else pg_bar();
  bf16x8 fa[TM], fb[TN];
  read_frags(fa, fb, 0);

  constexpr int NM = TM * TN;
  auto mma = [&](int i0, int i1) {
#pragma unroll
    for (int i = 0; i < NM; ++i)
      if (i >= i0 && i < i1)
        acc[i / TN][i % TN] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[i % TN], fa[i / TN],
                                                                       acc[i / TN][i % TN], 0, 0, 0);
  };
  // step s: MFMAs [0, H1) -- wait for step s + 1 + barrier -- the P DMA pieces of step
  // s + S - 1, each behind a share of MFMAs [H1, H2) -- step s + 1's fragment reads interleaved
  // with MFMAs [H2, NM)
  constexpr int H1 = NM / 2, H2 = NM * 3 / 4;
  constexpr int DQ = (H2 - H1 + P - 1) / P;

  int t = t_begin, kt = 0, slot = 0;
  for (int s = 0; s < NS; ++s) {
    const bool more = s + 1 < NS;
    mma(0, H1);
    if (more) {
      // issued so far: steps 0 .. min(s + S - 2, NS - 1); newer than s + 1:
      const int last = s + S - 2 < NS - 1 ? s + S - 2 : NS - 1;
      pg_wait_steps<P>(last - (s + 1));
      if constexpr (MODE > 0) {
        transform(t_x, kt_x, slot + 1 == S ? 0 : slot + 1);   // step s + 1, before publishing
        advance_x();
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      } else {
        pg_bar();
      }
    }
    const bool iss = s + S - 1 < NS;
    const int islot = slot == 0 ? S - 1 : slot - 1;      // slot of step s - 1, free now
#pragma unroll
    for (int q = 0; q < P; ++q) {
      if (iss) issue_piece(q, kt_issue, islot);
      mma(H1 + q * DQ, H1 + (q + 1) * DQ < H2 ? H1 + (q + 1) * DQ : H2);
    }
    if (iss) advance_issue();
    const int nslot = slot + 1 == S ? 0 : slot + 1;
    bf16x8 na[TM], nb[TN];
    read_frags(na, nb, nslot);
    mma(H2, NM);
    constexpr int NR = TM + TN;
    constexpr int NL = NM - H2;
    constexpr int RPM = (NR + NL - 1) / NL;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x100, RPM, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    }
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) fa[tm] = na[tm];
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) fb[tn] = nb[tn];
    if (++kt == KT) {
      epilogue(t);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      kt = 0;
      ++t;
    }
    slot = nslot;
  }
  if constexpr (STATS) {
    if (run && rgrp >= 0) flush(rgrp, 0);
  }
}

template <int BN, int WM, int S, int MODE>
constexpr int pg_lds_bytes() {
  // ring (A, B, per-wave coefficient copies, residual), DMA sink, statistics rows
  constexpr int slot = (PG_BM + BN) * 64 + (MODE > 0 ? PG_NW * 1024 : 0) + (MODE == 2 ? PG_BM * 64 : 0);
  return S * slot + PG_NW * 1024 + WM * 2 * BN * 4;
}

template <int BN, int WM, int S, bool STATS, bool GATHER, int MODE>
void pg_launch_k(const PgemmArgs& g, const PgemmPro& pro, int grid, hipStream_t st) {
  constexpr int bytes = pg_lds_bytes<BN, WM, S, MODE>();
  static_assert(bytes <= 160 * 1024, "LDS");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)pgemm_kernel<BN, WM, S, STATS, GATHER, MODE>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    attr = true;
  }
  hipLaunchKernelGGL((pgemm_kernel<BN, WM, S, STATS, GATHER, MODE>), dim3(grid), dim3(PG_NT), bytes,
                     st, g, pro);
}

// ring depth per (tile width, prologue mode): the deepest that fits 160 KB
template <int BN, int WM, int S0, int S1, int S2>
int pg_launch(const PgemmArgs& g, const PgemmPro& pro, int grid, hipStream_t st) {
  const bool stats = g.stats != nullptr, gather = g.stride != 1;
  if (pro.mode == 0) {
    if (stats) {
      if (gather) pg_launch_k<BN, WM, S0, true, true, 0>(g, pro, grid, st);
      else pg_launch_k<BN, WM, S0, true, false, 0>(g, pro, grid, st);
    } else {
      if (gather) pg_launch_k<BN, WM, S0, false, true, 0>(g, pro, grid, st);
      else pg_launch_k<BN, WM, S0, false, false, 0>(g, pro, grid, st);
    }
    return 1;
  }
  if (gather) return 0;
  if (pro.mode == 1) {
    if (stats) pg_launch_k<BN, WM, S1, true, false, 1>(g, pro, grid, st);
    else pg_launch_k<BN, WM, S1, false, false, 1>(g, pro, grid, st);
    return 1;
  }
  if constexpr (S2 > 0) {
    if (pro.mode == 2) {
      if (stats) pg_launch_k<BN, WM, S2, true, false, 2>(g, pro, grid, st);
      else pg_launch_k<BN, WM, S2, false, false, 2>(g, pro, grid, st);
      return 1;
    }
  }
  return 0;
}

// coef[g][0][c] = gamma * rsqrt(var + eps), coef[g][1][c] = beta - mean * scale, from the
// producer's per-group sums (same arithmetic as bn.hip) or its running statistics
__global__ __launch_bounds__(256) void pg_coef_kernel(PgemmPro p, int K) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= p.G * K) return;
  const int gi = i / K, c = i - gi * K;
  float mean, var;
  if (p.stats) {
    mean = p.stats[(size_t)gi * 2 * K + c] * p.inv_count;
    var = fmaxf(p.stats[(size_t)gi * 2 * K + K + c] * p.inv_count - mean * mean, 0.f);
  } else {
    mean = p.rmean[c];
    var = p.rvar[c];
  }
  const float sc = p.gamma[c] * rsqrtf(var + p.eps);
  p.coef[(size_t)gi * 2 * K + c] = sc;
  p.coef[(size_t)gi * 2 * K + K + c] = p.beta[c] - mean * sc;
}

int pg_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
  }
  return cus;
}

}  // namespace

// returns 0 when the shape / tile is not supported (caller falls back to igemm)
int pgemm_launch(const PgemmArgs& g_in, int bn, int grid, hipStream_t st, const PgemmPro* pro_in) {
  PgemmArgs g = g_in;
  PgemmPro pro{};
  if (pro_in) pro = *pro_in;
  if (g.K % 8 || g.N % 8 || g.M <= 0 || g.N <= 0 || g.K <= 0) return 0;
  if (g.stats && g.group_rows < PG_BM) return 0;           // a tile straddles <= 1 group boundary
  if (pro.mode) {
    if (g.stride != 1 || !pro.coef || pro.G < 1 || pro.group_rows < PG_BM) return 0;
    if (pro.mode == 2 && !pro.res) return 0;
  }
  const int ntiles = ((g.M + PG_BM - 1) / PG_BM) * ((g.N + bn - 1) / bn);
  // default grid: one block per CU (the caller's ``grid`` caps it: the two-stream step can leave
  // CUs to the other stream, whose kernels cannot share a CU with a 130-160 KB LDS block)
  if (grid <= 0) grid = pg_cus();
  if (grid > ntiles) grid = ntiles;
  if (pro.mode) {
    const int n = pro.G * g.K;
    hipLaunchKernelGGL(pg_coef_kernel, dim3((n + 255) / 256), dim3(256), 0, st, pro, g.K);
  }
  switch (bn) {
    case 256: return pg_launch<256, 2, 4, 3, 0>(g, pro, grid, st);
    case 128: return pg_launch<128, 4, 5, 4, 3>(g, pro, grid, st);
    case 64: return pg_launch<64, 8, 6, 5, 3>(g, pro, grid, st);
    default: return 0;
  }
}
