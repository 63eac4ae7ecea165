// Shared epilogue of the MFMA convolution kernels (igemm.hip, hconv.hip).
//
// The accumulator layout both main loops produce (swapped-operand 16x16x32 MFMA: lane l holds
// output pixel l&15 and four consecutive channels), the fused epilogue (bias, bf16 round,
// ghost-BN statistics, BN-backward sums, coalesced row stores) and the in-launch split-K
// reduction by the last-arriving slice.  Included into each kernel TU; everything is in an
// anonymous namespace.
#pragma once
#include "common.h"
#include "igemm.h"

namespace {

constexpr int BK = 64;          // k elements per stage (8 chunks of 8)
constexpr int NT = 256;         // threads

#ifdef MERCURY_STAMPS
// Diagnostic build only (-DMERCURY_STAMPS): per-block s_memtime at the phase boundaries of the
// register-staged body -- entry, first stage staged, main loop done, epilogue done -- written
// by thread 0 into a buffer no other code reads (bench/stamp_conv.py).
__device__ unsigned long long g_stamps[8192][12];   // [8..10]: epilogue sub-phases
#define MA_STAMP(i)                                                                         \
  do {                                                                                      \
    if (threadIdx.x == 0) {                                                                 \
      const int b_ = blockIdx.x + blockIdx.y * gridDim.x;                                   \
      if (b_ < 8192) g_stamps[b_][i] = __builtin_amdgcn_s_memtime();                       \
    }                                                                                       \
  } while (0)
// per-phase cycle sums over the main loop (thread 0): [4] load issue, [5] MFMA phase,
// [6] stage store (incl. the wait for its loads), [7] barrier
#define MA_LAP(slot, t)                                                                     \
  do {                                                                                      \
    const unsigned long long n_ = __builtin_amdgcn_s_memtime();                            \
    lap[slot] += n_ - t;                                                                    \
    t = n_;                                                                                 \
  } while (0)
#else
#define MA_STAMP(i) (void)0
#define MA_LAP(slot, t) (void)0
#endif

// XCD-aware tile order.  The dispatcher places workgroup b on XCD b % 8 and each XCD has its
// own 4 MB L2, so with tile = blockIdx.x, neighbouring output tiles -- which share the 3x3
// halo rows of their input and, across N tiles, the same input rows entirely -- land on
// different L2s.  Renumber so XCD x runs one contiguous range of tiles (bijective on [0, n)).
MA_DEV int xcd_tile(int b, int n) {
  const int per = n >> 3, rem = n & 7, x = b & 7;
  return x * per + min(x, rem) + (b >> 3);
}

template <int BM, int BN>
struct Smem {
  static constexpr int STAGE = (BM + BN) * BK;              // bf16 elements
  static constexpr int RED_BYTES = 16 * BN * 4 + BM * (BN + 8) * 2;  // stats + staged tile
  static constexpr int bytes(int stages) {
    return stages * STAGE * 2 > RED_BYTES ? stages * STAGE * 2 : RED_BYTES;
  }
};

// DPP sum over the 16 lanes of a row (quad xor1, quad xor2, half-mirror, mirror)
MA_DEV float row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  return v;
}

// ---------------------------------------------------------------- epilogue
// BN-backward helpers (same arithmetic as bn.hip so fused and standalone reductions agree)
// act'(out) != 0  <=>  act == none, or lo < out < hi: bounds from the uniform act once, so the
// per-element test is two compares, one uniform OR and one select -- a runtime act switch inside
// the unrolled element loop was if-converted into every activation form plus selects.  act ==
// none passes EVERY value (NaN and +-inf included), exactly like bn.hip's act_mask, so a
// diverging run is not hidden from the health checks by the fused reduction.
MA_DEV void bn_act_bounds(int act, float& lo, float& hi) {
  lo = act == 0 ? -__builtin_huge_valf() : 0.f;
  hi = act == 2 ? 6.f : __builtin_huge_valf();
}
// Forward clamp bounds: act == none clamps against NaN, which v_max/v_min_f32 ignore (they
// return the non-NaN operand), so the clamp is the identity and a NaN input stays NaN as in
// bn.hip's act_fwd; relu / relu6 clamp as act_fwd does.
MA_DEV void act_clamp_bounds(int act, float& lo, float& hi) {
  lo = act == 0 ? __builtin_nanf("") : 0.f;
  hi = act == 2 ? 6.f : (act == 0 ? __builtin_nanf("") : __builtin_huge_valf());
}
MA_DEV void bn_mean_rstd8(const float* stats, int ld, float inv_cnt, float eps, float (&mean)[8],
                          float (&rstd)[8]) {
  const float4 a = *(const float4*)stats, b = *(const float4*)(stats + 4);
  const float4 c = *(const float4*)(stats + ld), d = *(const float4*)(stats + ld + 4);
  const float s[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  const float ss[8] = {c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w};
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    mean[k] = s[k] * inv_cnt;
    rstd[k] = rsqrtf(fmaxf(ss[k] * inv_cnt - mean[k] * mean[k], 0.f) + eps);
  }
}

// Waves are laid out WM x WN (WM * WN = 4): 2 x 2 for the LDS-staged loops, 4 x 1 for the
// direct-A loop.  acc[tm][tn][j] =
//   OUT[m0 + wm*(BM/WM) + tm*16 + (lane&15)][n0 + wn*(BN/WN) + tn*16 + 4*(lane>>4) + j]
template <int BM, int BN, int WM>
using AccT = f32x4[BM / (16 * WM)][BN * WM / 64];

// output row of GEMM row ``row`` (identity unless a stride-2 dgrad parity class, EpiParams.rm_*)
MA_DEV int phys_row(const EpiParams& e, int row) {
  if (e.rm_hc == 0) return row;
  const int per = e.rm_hc * e.rm_wc;
  const int n = udiv24(row, per, 1.f / (float)per), rem = row - n * per;
  const int i = udiv24(rem, e.rm_wc, 1.f / (float)e.rm_wc), j = rem - i * e.rm_wc;
  return (n * e.rm_h + 2 * i + e.rm_ph) * e.rm_w + 2 * j + e.rm_pw;
}

template <int BM, int BN, int WM = 2>
MA_DEV void epilogue(AccT<BM, BN, WM>& acc, char* smem, const EpiParams& e, int M, int N,
                     int m0, int n0) {
  constexpr int WN = 4 / WM, TM = BM / (16 * WM), TN = BN / (16 * WN), LDT = BN + 8;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w / WN, wn = w % WN;
  const bool stats = e.stats != nullptr;
  const bool bw = e.bw_sums != nullptr;
  // stats: [WM][4][BN] per-wave-row partials (sum | sumsq | group-2 sum | group-2 sumsq),
  // each slot written by exactly one lane -- no LDS atomics, no zeroing; bw: [3][BN] sums
  float* red = (float*)smem;
  bf16* tile = (bf16*)(smem + 16 * BN * 4);        // [BM][LDT] staged output
  if (bw) {
    for (int i = tid; i < 3 * BN; i += NT) red[i] = 0.f;
  }
  // ghost-BN groups: a tile may straddle ONE group boundary (groups are >= BM rows), e.g. when
  // the per-image pixel count is odd (speech VGG 101x161); rows >= bnd go to group g + 1
  const int g0 = stats ? m0 / e.group_rows : 0;
  const int bnd = stats ? (g0 + 1) * e.group_rows : 0;
  const bool straddle = stats && bnd < m0 + BM && bnd < M;
  float4 bias[TN];
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) bias[tn] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (e.bias) {
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int nb = n0 + wn * (BN / WN) + tn * 16 + 4 * (lane >> 4);
      bias[tn] = *(const float4*)(e.bias + (nb < N ? nb : N - 4));
    }
  }
  __syncthreads();
  MA_STAMP(8);
  const int mrow = m0 + wm * (BM / WM) + (lane & 15);
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) {
    const int nl = wn * (BN / WN) + tn * 16 + 4 * (lane >> 4);
    float s[4] = {0.f, 0.f, 0.f, 0.f}, ss[4] = {0.f, 0.f, 0.f, 0.f};
    float s2[4] = {0.f, 0.f, 0.f, 0.f}, ss2[4] = {0.f, 0.f, 0.f, 0.f};
    const float bb[4] = {bias[tn].x, bias[tn].y, bias[tn].z, bias[tn].w};
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
      const int ml = wm * (BM / WM) + tm * 16 + (lane & 15);
      bf16x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = f2bf(acc[tm][tn][j] + bb[j]);
      *(bf16x4*)(tile + ml * LDT + nl) = o;   // one 8-byte LDS write per lane
      const int row = mrow + tm * 16;
      if (stats) {
        if (!straddle) {
          // rows past M masked by a multiply, not an exec-mask branch per fragment
          const float msk = row < M ? 1.f : 0.f;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float f = bf2f(o[j]) * msk;
            s[j] += f;
            ss[j] += f * f;
          }
        } else if (row < M) {
          if (row < bnd) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float f = bf2f(o[j]);
              s[j] += f;
              ss[j] += f * f;
            }
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float f = bf2f(o[j]);
              s2[j] += f;
              ss2[j] += f * f;
            }
          }
        }
      }
    }
    if (stats) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s[j] = row16_sum(s[j]);
        ss[j] = row16_sum(ss[j]);
      }
      if (straddle) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          s2[j] = row16_sum(s2[j]);
          ss2[j] = row16_sum(ss2[j]);
        }
      }
      if ((lane & 15) == 0) {
        float* r = red + wm * 4 * BN + nl;
        *(float4*)r = make_float4(s[0], s[1], s[2], s[3]);
        *(float4*)(r + BN) = make_float4(ss[0], ss[1], ss[2], ss[3]);
        if (straddle) {
          *(float4*)(r + 2 * BN) = make_float4(s2[0], s2[1], s2[2], s2[3]);
          *(float4*)(r + 3 * BN) = make_float4(ss2[0], ss2[1], ss2[2], ss2[3]);
        }
      }
    }
  }
  MA_STAMP(9);
  __syncthreads();
  if (stats) {
    for (int gi = 0; gi < (straddle ? 2 : 1); ++gi) {
      float* dst = MA_SPREAD(e.stats + (size_t)(g0 + gi) * 2 * e.stats_ld);
      for (int i = tid; i < BN; i += NT) {
        const int col = n0 + i;
        if (col < N) {
          float a = 0.f, b = 0.f;
#pragma unroll
          for (int q = 0; q < WM; ++q) {
            a += red[(q * 4 + 2 * gi) * BN + i];
            b += red[(q * 4 + 2 * gi + 1) * BN + i];
          }
          atomicAdd(dst + col, a);
          atomicAdd(dst + e.stats_ld + col, b);
        }
      }
    }
  }
  // coalesced 16-byte row stores from the staged tile.  NT is a multiple of CPR, so every
  // thread keeps ONE 8-column chunk for the whole loop (its BN constants load once).
  constexpr int CPR = BN / 8;
  const int ch = tid % CPR;
  const int colc = n0 + ch * 8;
  float mean[8], rstd[8], mean2[8], rstd2[8], sdz[8], sx[8], sx2[8];
  const bool two = bw && e.bw_y2 != nullptr;
  float alo, ahi;
  bn_act_bounds(e.bw_act, alo, ahi);
  const bool pass = e.bw_act == 0;
  if (bw) {
#pragma unroll
    for (int k = 0; k < 8; ++k) sdz[k] = sx[k] = sx2[k] = mean2[k] = 0.f, rstd2[k] = 1.f;
    const int cc = colc < N ? colc : 0;
    bn_mean_rstd8(e.bw_stats + cc, e.ldo, e.bw_inv_count, e.bw_eps, mean, rstd);
    if (two) bn_mean_rstd8(e.bw_stats2 + cc, e.ldo, e.bw_inv_count, e.bw_eps, mean2, rstd2);
  }
  MA_STAMP(10);
  for (int i = tid; i < BM * CPR; i += NT) {
    const int rl = i / CPR;
    const int row = m0 + rl, col = colc;
    if (row >= M || col >= N) continue;
    bf16x8 v = *(const bf16x8*)(tile + rl * LDT + ch * 8);
    const size_t off = (size_t)phys_row(e, row) * e.ldo + col;
    bf16* dst = e.out + off;
    if (e.accumulate) {
      const bf16x8 o = *(const bf16x8*)dst;
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = f2bf(bf2f(v[k]) + bf2f(o[k]));
    }
    *(bf16x8*)dst = v;
    if (bw) {
      const bf16x8 ao = *(const bf16x8*)(e.bw_out + off);
      const bf16x8 ay = *(const bf16x8*)(e.bw_y + off);
      bf16x8 ay2;
      if (two) ay2 = *(const bf16x8*)(e.bw_y2 + off);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float ok = bf2f(ao[k]);
        const float dz = (pass || (ok > alo && ok < ahi)) ? bf2f(v[k]) : 0.f;
        sdz[k] += dz;
        sx[k] += dz * (bf2f(ay[k]) - mean[k]) * rstd[k];
        if (two) sx2[k] += dz * (bf2f(ay2[k]) - mean2[k]) * rstd2[k];
      }
    }
  }
  if (bw) {
    // lanes ch, ch+CPR, ... of a wave share the chunk: butterfly, then one LDS atomic per
    // (wave, column), then one global atomic per column per block
#pragma unroll
    for (int k = 0; k < 8; ++k) {
#pragma unroll
      for (int o = CPR; o < 64; o <<= 1) {
        sdz[k] += __shfl_xor(sdz[k], o, 64);
        sx[k] += __shfl_xor(sx[k], o, 64);
        if (two) sx2[k] += __shfl_xor(sx2[k], o, 64);
      }
    }
    if (lane < CPR) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        atomicAdd(&red[ch * 8 + k], sdz[k]);
        atomicAdd(&red[BN + ch * 8 + k], sx[k]);
        if (two) atomicAdd(&red[2 * BN + ch * 8 + k], sx2[k]);
      }
    }
    __syncthreads();
    // replica (row tile % SUMS_R) of the [SUMS_R][3][ldo] sums (igemm.h)
    float* sums = e.bw_sums + (size_t)((m0 / BM) % SUMS_R) * 3 * e.ldo;
    for (int i = tid; i < BN; i += NT) {
      const int col = n0 + i;
      if (col < N) {
        atomicAdd(sums + col, red[i]);
        atomicAdd(sums + e.ldo + col, red[BN + i]);
        if (two) atomicAdd(sums + 2 * e.ldo + col, red[2 * BN + i]);
      }
    }
  }
}

// Split-K: every K-slice block writes its fp32 partial tile (fragment order, 16 B per lane,
// fully coalesced) behind the slab's tile-counter header; the LAST block to arrive on a tile
// sums all slices and runs the epilogue in the same launch (no reducer kernel, no extra launch
// in the step graph).  Hand-off (cdna_hip_programming.md §6 Guideline 16, R1 form): partials are
// stored write-through (buffer store, sc1) and drained by every wave before the workgroup
// barrier, one lane takes a relaxed agent-scope ticket; the last arriver reads the other slices
// with sc1 loads only -- no L2 write-back fence per block, correct for any XCD placement.  The
// counter is reset by the last arriver (slabs are zero-initialised at allocation).
constexpr int SEM_INTS = 1024;   // tile counters at the head of the slab (4 KB)

template <int BM, int BN, int WM = 2>
MA_DEV void finish(AccT<BM, BN, WM>& acc, char* smem, const EpiParams& e, int M, int N,
                   int m0, int n0, int bx, int by, int gx, int gy) {
  constexpr int TM = BM / (16 * WM), TN = BN * WM / 64;
  if (e.slab) {
    const int ntiles = gx;
    const int splits = gy;
    int* sem = (int*)e.slab;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(e.slab + SEM_INTS), 0, 0x7fffffff,
                                                      0x00020000);
    const int tile_bytes = TM * TN * NT * 16;
    const int mine = (by * ntiles + bx) * tile_bytes + threadIdx.x * 16;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[tm][tn]), rs,
                                               mine + (tm * TN + tn) * NT * 16, 0, 16 /*sc1*/);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains
    int* flag = (int*)smem;
    __syncthreads();
    if (threadIdx.x == 0) {
      const int old = __hip_atomic_fetch_add(&sem[bx], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == splits - 1;
      if (last) __hip_atomic_store(&sem[bx], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag[0] = last;
    }
    __syncthreads();
    if (!flag[0]) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // keep the sc1 loads below the ticket
    for (int sp = 0; sp < splits; ++sp) {
      if (sp == by) continue;
      const int base = (sp * ntiles + bx) * tile_bytes + threadIdx.x * 16;
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] += __builtin_bit_cast(
              f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, base + (tm * TN + tn) * NT * 16, 0,
                                                           16 /*sc1*/));
    }
    __syncthreads();   // flag read by every wave before the epilogue reuses smem
  }
  epilogue<BM, BN, WM>(acc, smem, e, M, N, m0, n0);
}

}  // namespace
