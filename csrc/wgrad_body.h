// Weight-gradient implicit GEMM body (device code shared by wgrad.hip's standalone kernel
// and igemm.hip's dgrad+wgrad pair launch).  See wgrad.hip for the algorithm.
#pragma once
#include "common.h"
#include "igemm.h"

namespace wgb {
constexpr int WG_NT = 256;
constexpr int WG_BKP = 64;  // pixels per stage
constexpr int WG_SEM_INTS = 1024;   // tile counters at the head of a wgrad slab (4 KB)

typedef short short4_t __attribute__((ext_vector_type(4)));

MA_DEV bf16x4 tr_read(const bf16* p) {
  short4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) short4_t*)(p));
  return __builtin_bit_cast(bf16x4, v);
}

template <int BM, int BN>
struct WgSmem {
  static constexpr int STAGE = WG_BKP * ((BM + 16) + (BN + 16));   // bf16 elements
  static constexpr int BYTES = 2 * STAGE * 2;
};

// One (column tile bx, pixel split by) of the weight-gradient GEMM; gy = number of splits.
// PF: stages in flight in registers -- 2 where the extra register set fits (64-wide tiles),
// 1 for 128 x 128 (the second set spilled)
template <int BM, int BN, int PF = (BM * BN <= 64 * 128 ? 2 : 1)>
MA_DEV void wgrad_body(const bf16* __restrict__ dy, const bf16* __restrict__ x, const WgradGeom& g,
                       float* __restrict__ dw, int ptiles_per_split, bf16* smem, int bx, int by,
                       int gy) {
  constexpr int NT = WG_NT, BKP = WG_BKP;
  constexpr int LDA = BM + 16, LDB = BN + 16;
  constexpr int STAGE = WgSmem<BM, BN>::STAGE;
  constexpr int TM = BM / 32, TN = BN / 32;
  constexpr int ACH = BM / 8, BCH = BN / 8;          // chunks per row
  constexpr int AR = BKP * ACH / NT, BR = BKP * BCH / NT;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int C8 = g.C >> 3;
  const int Kc = g.R * g.S * C8;                       // reduction-free column chunks
  const int ncols = Kc * 8;
  const int ntn = (ncols + BN - 1) / BN;
  const int mt = bx / ntn, nt = bx - mt * ntn;
  const int m0 = mt * BM, n0 = nt * BN;
  const int npix = g.N * g.P * g.Q;
  const int ptiles = (npix + BKP - 1) / BKP;
  const int pt0 = by * ptiles_per_split;
  const int pt1 = min(ptiles, pt0 + ptiles_per_split);

  // fixed column chunk per thread for the x tile
  const int bcc = tid % BCH;
  const int jc = n0 / 8 + bcc;
  int xr = 0, xs = 0, xc8 = 0;
  const bool jval = jc < Kc;
  if (jval) {
    const int rs = jc / C8;
    xc8 = jc - rs * C8;
    xr = rs / g.S;
    xs = rs - xr * g.S;
  }
  const int acc_ = tid % ACH;

  // Operands through buffer resources with 32-bit byte offsets: an invalid row (padding tap,
  // past the pixel range, past K) gets an offset beyond the resource and loads zeros -- no
  // zero-page select, no exec-masked branch, no 64-bit address math per row (the per-row
  // 64-bit multiplies and the two pixel divisions per stage made the loop VALU-bound).
  const auto rdy = __builtin_amdgcn_make_buffer_rsrc((void*)dy, 0, npix * g.K * 2, 0x00020000);
  const auto rx = __builtin_amdgcn_make_buffer_rsrc((void*)x, 0, g.N * g.H * g.W * g.C * 2,
                                                    0x00020000);
  constexpr unsigned BAD = 0x80000000u;
  // A (dy) rows: pixel pixA + i * (NT / ACH), channel chunk k; advanced by BKP pixels a stage
  const int k = m0 + acc_ * 8;
  int pixA = pt0 * BKP + tid / ACH;
  // B (x) rows: the source pixel's (n, p, q), advanced by BKP pixels a stage without a division
  // (q += BKP % Q, p += BKP / Q, carries); a 1x1 stride-1 conv reads x at the dy pixel itself
  const bool pw = g.R == 1 && g.S == 1 && g.stride == 1 && g.pad == 0;
  const int aq = BKP % g.Q, ap = BKP / g.Q;
  int pixB = pt0 * BKP + tid / BCH;
  int bn_[BR], bp_[BR], bq_[BR];
#pragma unroll
  for (int i = 0; i < BR; ++i) {
    const int pix = pixB + i * (NT / BCH);
    const int pq = g.P * g.Q;
    bn_[i] = pix / pq;
    const int rem = pix - bn_[i] * pq;
    bp_[i] = rem / g.Q;
    bq_[i] = rem - bp_[i] * g.Q;
  }
  // stage loads into a register set; a stage past this split's range loads zeros, so every
  // trip issues the same number of loads and hipcc's counted vmcnt stays exact
  auto load_stage = [&](int pt, u32x4 (&ra)[AR], u32x4 (&rb)[BR]) {
    const bool live = pt < pt1;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int pix = pixA + i * (NT / ACH);
      const bool ok = live && pix < npix && k < g.K;
      ra[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                            rdy, ok ? (unsigned)(pix * g.K + k) * 2u : BAD, 0, 0));
    }
    pixA += BKP;
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      unsigned off;
      bool ok;
      if (pw) {                          // kernel-uniform
        const int pix = pixB + i * (NT / BCH);
        ok = live && jval && pix < npix;
        off = (unsigned)(pix * g.C + xc8 * 8) * 2u;
      } else {
        const int h = bp_[i] * g.stride - g.pad + xr, ww = bq_[i] * g.stride - g.pad + xs;
        ok = live && jval && bn_[i] < g.N && (unsigned)h < (unsigned)g.H &&
             (unsigned)ww < (unsigned)g.W;
        off = (unsigned)(((bn_[i] * g.H + h) * g.W + ww) * g.C + xc8 * 8) * 2u;
        int q = bq_[i] + aq, p = bp_[i] + ap, n = bn_[i];
        if (q >= g.Q) {
          q -= g.Q;
          ++p;
        }
        while (p >= g.P) {
          p -= g.P;
          ++n;
        }
        bn_[i] = n;
        bp_[i] = p;
        bq_[i] = q;
      }
      rb[i] = __builtin_bit_cast(u32x4,
                                 __builtin_amdgcn_raw_buffer_load_b128(rx, ok ? off : BAD, 0, 0));
    }
    pixB += BKP;
  };
  auto store_stage = [&](int buf, const u32x4 (&ra)[AR], const u32x4 (&rb)[BR]) {
    bf16* a = smem + buf * STAGE;
    bf16* b = a + BKP * LDA;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int row = tid / ACH + i * (NT / ACH);
      *(u32x4*)(a + row * LDA + acc_ * 8) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int row = tid / BCH + i * (NT / BCH);
      *(u32x4*)(b + row * LDB + bcc * 8) = rb[i];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g4 = lane >> 4, li = lane & 15;
  const int tq = li >> 2, tp = li & 3;
  auto mma = [&](int buf) {
    const bf16* a = smem + buf * STAGE;
    const bf16* b = a + BKP * LDA;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[TM], fb[TN];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int row = kk * 32 + 16 * h + 4 * g4 + tq;
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
          const bf16x4 v = tr_read(a + row * LDA + wm * (BM / 2) + tm * 16 + 4 * tp);
#pragma unroll
          for (int e = 0; e < 4; ++e) fa[tm][4 * h + e] = v[e];
        }
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
          const bf16x4 v = tr_read(b + row * LDB + wn * (BN / 2) + tn * 16 + 4 * tp);
#pragma unroll
          for (int e = 0; e < 4; ++e) fb[tn][4 * h + e] = v[e];
        }
      }
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[tm], fb[tn], acc[tm][tn], 0, 0, 0);
    }
  };
  if (pt0 < pt1 && PF == 1) {
    u32x4 ra[AR], rb[BR];
    load_stage(pt0, ra, rb);
    store_stage(0, ra, rb);
    __syncthreads();
    int buf = 0;
    for (int pt = pt0; pt < pt1; ++pt) {
      const bool more = pt + 1 < pt1;
      if (more) load_stage(pt + 1, ra, rb);
      mma(buf);
      if (more) store_stage(buf ^ 1, ra, rb);
      __syncthreads();
      buf ^= 1;
    }
  } else if (pt0 < pt1) {
    // two stages in flight in registers (the train-batch wgrad is latency-bound: a 64-pixel
    // stage is ~8 MFMAs per wave, far shorter than a memory round trip), LDS double-buffered;
    // unrolled by two so each register set is named statically
    u32x4 ra0[AR], rb0[BR], ra1[AR], rb1[BR];
    load_stage(pt0, ra0, rb0);
    store_stage(0, ra0, rb0);
    load_stage(pt0 + 1, ra1, rb1);
    __syncthreads();
    for (int pt = pt0; pt < pt1; pt += 2) {
      load_stage(pt + 2, ra0, rb0);      // LDS 0 holds stage pt, ra1 stage pt + 1
      mma(0);
      if (pt + 1 >= pt1) break;
      store_stage(1, ra1, rb1);
      __syncthreads();
      load_stage(pt + 3, ra1, rb1);      // LDS 1 holds stage pt + 1, ra0 stage pt + 2
      mma(1);
      if (pt + 2 >= pt1) break;
      store_stage(0, ra0, rb0);
      __syncthreads();
    }
  }

  // Split-K over pixels with a slab (large pixel counts: many splits, no contended atomics):
  // each split writes its fp32 partial tile write-through (16 B per lane, coalesced), takes a
  // ticket on the tile's counter, and the LAST split to arrive sums the others and stores dW
  // (same hand-off as the dgrad split-K, conv_epi.h finish()).  Without a slab, splits add
  // into dW with fp32 atomics.
  bool atomic = gy > 1;
  if (atomic && g.slab != nullptr) {
    atomic = false;
    const int ntiles = (g.K + BM - 1) / BM * ntn;
    int* sem = (int*)g.slab;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(g.slab + WG_SEM_INTS), 0,
                                                      0x7fffffff, 0x00020000);
    constexpr int tile_bytes = TM * TN * NT * 16;
    const int mine = (by * ntiles + bx) * tile_bytes + tid * 16;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[tm][tn]), rs,
                                               mine + (tm * TN + tn) * NT * 16, 0, 16 /*sc1*/);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains
    int* flag = (int*)smem;
    __syncthreads();                                     // (also: the last stage's LDS reads)
    if (tid == 0) {
      const int old = __hip_atomic_fetch_add(&sem[bx], 1, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == gy - 1;
      if (last) __hip_atomic_store(&sem[bx], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag[0] = last;
    }
    __syncthreads();
    if (!flag[0]) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // keep the sc1 loads below the ticket
    for (int sp = 0; sp < gy; ++sp) {
      if (sp == by) continue;
      const int base = (sp * ntiles + bx) * tile_bytes + tid * 16;
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] += __builtin_bit_cast(
              f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, base + (tm * TN + tn) * NT * 16, 0,
                                                           16 /*sc1*/));
    }
  }
  const int RSCr = g.R * g.S * g.Creal;
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) {
    const int col = n0 + wn * (BN / 2) + tn * 16 + li;
    if (col >= ncols) continue;
    const int rs = col / g.C, c = col - rs * g.C;
    if (c >= g.Creal) continue;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = m0 + wm * (BM / 2) + tm * 16 + g4 * 4 + j;
        if (k >= g.K) continue;
        float* dst = dw + (size_t)k * RSCr + rs * g.Creal + c;
        if (atomic) atomicAdd(dst, acc[tm][tn][j]);
        else *dst = acc[tm][tn][j];
      }
    }
  }
}

// grid decomposition shared by the standalone and the pair launches
inline void wg_grid(const WgradGeom& g, int bm, int bn, int splits, int& gx, int& per, int& gy) {
  const int ncols = g.R * g.S * g.C;
  const int mtiles = (g.K + bm - 1) / bm, ntiles = (ncols + bn - 1) / bn;
  const int ptiles = (g.N * g.P * g.Q + WG_BKP - 1) / WG_BKP;
  splits = splits < 1 ? 1 : (splits > ptiles ? ptiles : splits);
  per = (ptiles + splits - 1) / splits;
  gy = (ptiles + per - 1) / per;
  gx = mtiles * ntiles;
}

// bytes of the slab a split launch needs (counters + one partial tile per (split, tile))
inline size_t wg_slab_bytes(int gx, int gy, int bm, int bn) {
  return (size_t)WG_SEM_INTS * 4 + (size_t)gx * gy * bm * bn * 4;
}
}  // namespace wgb
