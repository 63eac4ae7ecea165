// Implicit-GEMM convolution on MFMA (gfx950): forward and data-gradient.
//
// Replaces cuDNN/MIOpen conv for the reference's ResNet/VGG/MobileNet stacks
// (`pytorch_model.py:19-36,72-97`).  One "NT" GEMM kernel serves both
// directions:
//
//   OUT[m][n] = sum_k A[m][k] * B[n][k]          m = pixel, n = channel,
//                                                k = (r, s, c) with c fastest
//
//   forward : A = im2col(x), rows are OUTPUT pixels, h = p*stride - pad + r
//   dgrad   : A = col2im-gather(dy), rows are INPUT pixels, p = (h + pad - r)/stride
//             when divisible (TRANS=true); B = the weight transposed to [C][R][S][K]
//
// Both operands are K-contiguous in HBM (NHWC activations, [N][K] weights), so
// one 16-byte load = one (pixel, 8-channel) chunk = exactly the 8 bf16 a lane
// feeds to v_mfma_f32_16x16x32_bf16 (lane l: row l&15, k = 8*(l>>4)..+7).
//
// The MFMA is issued with the operands SWAPPED (weights as the "A" input, pixels
// as "B"), so the accumulator comes out transposed: lane l holds output pixel
// l&15 and FOUR CONSECUTIVE CHANNELS 4*(l>>4)..+3 -- 8 contiguous bytes of the
// NHWC output.  The epilogue therefore stores straight from registers (no LDS
// staging pass), and BN statistics reduce across the 16 pixel lanes with four
// DPP row operations (cdna_hip_programming.md §3: choose the product orientation
// so later consumers see the layout they want).
//
// Main loop: 256 threads = 4 waves (2x2), BK = 64 per stage, register-staged double buffer
// (stage t+1 loads issued before stage t's MFMAs, one barrier per stage).  (An LDS-DMA ring
// variant was A/B'd slower on every conv shape of the step and removed in round 3; the 1x1
// convs that gain from an LDS-DMA pipeline run on the persistent pointwise GEMM, pgemm.hip.)
// LDS rows are XOR-swizzled (chunk c of row r lives at c ^ (r&7)).  All address math
// is 32-bit (per-row base offsets + one uniform per-tap offset), padding chunks read
// a zero page.  Split-K writes fp32 partial tiles in fragment order (16 B per lane,
// fully coalesced); the last-arriving slice of each tile reduces them and runs the
// same epilogue inside the launch (see finish()).

#include "conv_epi.h"
#include "wgrad_body.h"

namespace {


__device__ __attribute__((aligned(16))) bf16 g_zero_page[64];

MA_DEV int swz(int row, int chunk) { return chunk ^ (row & 7); }

// 256 x 128 tiles (the B = 320 scoring convs): 128 fp32 accumulators per lane and 96 KB of
// stages -- one block per CU, every register available to it
template <int BM, int BN>
constexpr int nt_occ() { return BM * BN >= 256 * 128 ? 1 : 2; }


// ---------------------------------------------------------------- A-row gather helpers
// (plain scalars per row -- a struct holding the per-row arrays was demoted to scratch
// by hipcc, which turned every gather into a scratch load + vmcnt(0))
template <bool TRANS>
MA_DEV void row_init(const ConvGeom& g, int m, int& off, int& h, int& w) {
  const int pq = g.RP * g.RQ;
  const int mm = m < g.M ? m : 0;
  const int n = udiv24(mm, pq, 1.f / (float)pq), rem = mm - n * pq;
  const int p = udiv24(rem, g.RQ, 1.f / (float)g.RQ), q = rem - p * g.RQ;
  off = m < g.M ? n * g.SH * g.SW : -1;
  h = TRANS ? p + g.pad : p * g.stride - g.pad;
  w = TRANS ? q + g.pad : q * g.stride - g.pad;
}

// element offset of (row, tap r/s, channel chunk c8) or -1 for a zero chunk.  Branch-free:
// the bounds tests become compares + one select, so the per-row gather of a stage is straight-
// line VALU and every load issues unconditionally (a divergent branch per row made hipcc wrap
// each load in exec-mask save/restore and re-derive the zero-page address in every branch).
template <bool TRANS>
MA_DEV int row_at(const ConvGeom& g, int off, int h, int w, int r, int s, int c8) {
  int hh, ww;
  bool ok = off >= 0;
  if (TRANS) {
    const int hp = h - r, wp = w - s;
    if (g.stride == 2) {                 // kernel-uniform: scalar branch
      ok = ok && ((hp | wp) & 1) == 0;
      hh = hp >> 1;                      // arithmetic shift keeps negatives negative
      ww = wp >> 1;
    } else {
      hh = hp;
      ww = wp;
    }
  } else {
    hh = h + r;
    ww = w + s;
  }
  ok = ok && (unsigned)hh < (unsigned)g.SH && (unsigned)ww < (unsigned)g.SW;
  const int o = (off + hh * g.SW + ww) * g.SC + c8 * 8;
  return ok ? o : -1;
}

// Register-staged loop addressing (see igemm_nt_body): element offset of the row's source
// pixel at tap (0, 0), the uniform offset of tap (r, s) from it, and the tap's bounds test.
// forward: +(r*SW + s); dgrad stride 1: -(r*SW + s); dgrad stride 2: -((r>>1)*SW + (s>>1)),
// valid only when the row's parity matches the tap's (then (h - r) >> 1 == (h >> 1) - (r >> 1)).
template <bool TRANS>
MA_DEV int row_base(const ConvGeom& g, int off, int h, int w) {
  if (TRANS && g.stride == 2) return (off + (h >> 1) * g.SW + (w >> 1)) * g.SC;
  return (off + h * g.SW + w) * g.SC;
}

template <bool TRANS>
MA_DEV int tap_offset(const ConvGeom& g, int r, int s) {
  if (!TRANS) return (r * g.SW + s) * g.SC;
  if (g.stride == 2) return -((r >> 1) * g.SW + (s >> 1)) * g.SC;
  return -(r * g.SW + s) * g.SC;
}

template <bool TRANS>
MA_DEV bool tap_ok(const ConvGeom& g, int h, int w, int r, int s) {
  if (!TRANS) return (unsigned)(h + r) < (unsigned)g.SH && (unsigned)(w + s) < (unsigned)g.SW;
  const int hp = h - r, wp = w - s;
  if (g.stride == 2)   // kernel-uniform: scalar branch
    return ((hp | wp) & 1) == 0 && (unsigned)(hp >> 1) < (unsigned)g.SH &&
           (unsigned)(wp >> 1) < (unsigned)g.SW;
  return (unsigned)hp < (unsigned)g.SH && (unsigned)wp < (unsigned)g.SW;
}

// k-chunk -> (r, s, c8) cursor.  When C/8 is a multiple of 8 a 64-deep stage lies in one
// filter tap, so the tap advances incrementally (no division in the loop).  Otherwise the
// stage base is decoded once (uniform) and each lane steps its <= 7 extra chunks forward;
// the tap split r = rs / S uses an exact float reciprocal (rs <= R*S <= 49).
struct KCursor {
  int tr, ts, tc;
  bool fast;
  MA_DEV void init(const ConvGeom& g, int kt0) {
    const int C8 = g.SC >> 3;
    fast = (C8 & 7) == 0;
    tr = ts = tc = 0;
    if (fast) {
      const int k0c = kt0 * 8;
      const int rs = k0c / C8;
      tc = k0c - rs * C8;
      tr = rs / g.S;
      ts = rs - tr * g.S;
    }
  }
  // decode the chunk `lcc` (0..7) of stage kt and advance after the last use
  MA_DEV void decode(const ConvGeom& g, int kt, int lcc, int& r, int& s, int& c8, bool& kval) const {
    const int kc = kt * 8 + lcc;
    kval = kc < g.Kc;
    if (fast) {
      r = tr;
      s = ts;
      c8 = tc + lcc;
    } else {
      const int C8 = g.SC >> 3;
      const int k0 = kt * 8;                       // uniform
      int rs = k0 / C8;
      c8 = k0 - rs * C8 + lcc;
      while (c8 >= C8) {                           // <= 8 / C8 trips
        c8 -= C8;
        ++rs;
      }
      r = (int)(((float)rs + 0.5f) * (1.f / (float)g.S));
      s = rs - r * g.S;
    }
  }
  MA_DEV void advance(const ConvGeom& g) {
    if (!fast) return;
    tc += 8;
    if (tc == (g.SC >> 3)) {
      tc = 0;
      if (++ts == g.S) {
        ts = 0;
        ++tr;
      }
    }
  }
};

template <int BM, int BN>
MA_DEV void mma_stage(const bf16* a, const bf16* b, f32x4 (&acc)[BM / 32][BN / 32], int lane,
                      int wm, int wn) {
  constexpr int TM = BM / 32, TN = BN / 32;
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int chunk = kk * 4 + (lane >> 4);
    bf16x8 fa[TM], fb[TN];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
      const int row = wm * (BM / 2) + tm * 16 + (lane & 15);
      fa[tm] = *(const bf16x8*)(a + row * BK + swz(row, chunk) * 8);
    }
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int row = wn * (BN / 2) + tn * 16 + (lane & 15);
      fb[tn] = *(const bf16x8*)(b + row * BK + swz(row, chunk) * 8);
    }
    // swapped operands: weights as the MFMA "A", pixels as "B" -> transposed accumulator
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[tn], fa[tm], acc[tm][tn], 0, 0, 0);
  }
}

// ---------------------------------------------------------------- register-staged loop
// One (tile bx, K-split by) of the NT GEMM; gx tiles x gy splits in the launch.
// PRO: BN-apply + activation of the A operand between the global load and the LDS write
// (ProParams in igemm.h).  Everything it needs for the chunk staged next -- the 8 channels'
// statistics / gamma / beta, which rows are padding, where the activation is kept -- is loaded
// or computed in load_stage, so it is in flight under the MFMA phase like the tile itself.
template <int BM, int BN, bool TRANS, bool PRO = false, int PF = 1>
MA_DEV void igemm_nt_body(const bf16* __restrict__ src, const bf16* __restrict__ wt,
                          const ConvGeom& g, const EpiParams& e, int ktiles_per_split, char* smem,
                          int bx, int by, int gx, int gy, const ProParams& pro) {
  constexpr int TM = BM / 32, TN = BN / 32;
  constexpr int AR = BM / 32, BR = BN / 32;  // rows per thread for A / B staging
  bf16* sA = (bf16*)smem;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int ntn = (g.Ncols + BN - 1) / BN;
  const int mt = bx / ntn, nt = bx - mt * ntn;
  const int m0 = mt * BM, n0 = nt * BN;
  MA_STAMP(0);
  const int ktiles = (g.Kc + 7) / 8;
  const int kt0 = by * ktiles_per_split;
  const int kt1 = min(ktiles, kt0 + ktiles_per_split);
  const int Kelems = g.Kc * 8;
  const int cc = tid & 7;

  // A rows: the source offset of tap (0, 0) is computed once per row (abase), so a stage's
  // gather is  abase + uniform tap offset  plus two bounds tests -- no per-row multiplies
  // (stamps: the per-row multiply-heavy row_at was ~45 % of each stage's cycles).  A row
  // past M gets an out-of-range h, so its bounds test always fails.
  int abase[AR], ah[AR], aw[AR];
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    int off;
    row_init<TRANS>(g, m0 + (tid >> 3) + 32 * i, off, ah[i], aw[i]);
    abase[i] = row_base<TRANS>(g, off, ah[i], aw[i]);
    if (off < 0) ah[i] = -(1 << 28);
  }
  int boff[BR];
  const int ldb = g.ldb ? g.ldb : Kelems;
#pragma unroll
  for (int i = 0; i < BR; ++i) {
    const int n = n0 + (tid >> 3) + 32 * i;
    boff[i] = n < g.Ncols ? n * ldb : -1;
  }
  KCursor kc;
  kc.init(g, kt0);
  const bf16* zp = g.zero;

  // prologue state for the chunk in flight (PRO only; dead code otherwise)
  float4 pst[8];
  int pz = 0;
  int pko[AR];
  u32x4 prs[AR];       // residual chunks (pro.res)
  const float* pbase = nullptr;
  if constexpr (PRO) {
    const int grp = m0 / pro.group_rows;
    pbase = pro.stats ? pro.stats + (size_t)grp * 2 * g.SC : nullptr;
  }
  auto load_stage = [&](int kt, u32x4 (&ra)[AR], u32x4 (&rb)[BR]) {
    int r, s, c8;
    bool kval;
    kc.decode(g, kt, cc, r, s, c8, kval);
    kc.advance(g);
    kval = kval && kt < kt1;       // a prefetch past this split's range loads zeros
    bool keep = false;
    if constexpr (PRO) {
      const int ch = kval ? c8 * 8 : 0;
      const float* m0p = pbase ? pbase + ch : pro.rmean + ch;
      const float* v0p = pbase ? pbase + g.SC + ch : pro.rvar + ch;
      pst[0] = *(const float4*)m0p;
      pst[1] = *(const float4*)(m0p + 4);
      pst[2] = *(const float4*)v0p;
      pst[3] = *(const float4*)(v0p + 4);
      pst[4] = *(const float4*)(pro.gamma + ch);
      pst[5] = *(const float4*)(pro.gamma + ch + 4);
      pst[6] = *(const float4*)(pro.beta + ch);
      pst[7] = *(const float4*)(pro.beta + ch + 4);
      keep = pro.keep != nullptr && nt == 0 && kval && r * g.S + s == pro.keep_tap;
      pz = 0;
    }
    const int toff = tap_offset<TRANS>(g, r, s) + c8 * 8;
    // B chunk: the k chunk itself, or (parity class) the real weight tap of virtual tap (r, s)
    const int bch = g.trb < 0 ? kt * 8 + cc
                              : ((g.trb - 2 * r) * g.tS + (g.tsb - 2 * s)) * (g.SC >> 3) + c8;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const bool ok = kval && tap_ok<TRANS>(g, ah[i], aw[i], r, s);
      const int o = abase[i] + toff;
      ra[i] = *(const u32x4*)(ok ? src + o : zp);   // select, not a branch around the gather
      if constexpr (PRO) {
        pz |= (ok ? 0 : 1) << i;
        pko[i] = keep && ok ? o : -1;
        if (pro.res != nullptr) prs[i] = *(const u32x4*)(ok ? pro.res + o : zp);
      }
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const bool ok = kval && boff[i] >= 0;
      rb[i] = *(const u32x4*)(ok ? wt + boff[i] + bch * 8 : zp);
    }
  };
  auto store_stage = [&](int buf, u32x4 (&ra)[AR], const u32x4 (&rb)[BR]) {
    bf16* a = sA + buf * Smem<BM, BN>::STAGE;
    bf16* b = a + BM * BK;
    if constexpr (PRO) {
      const float mv[8] = {pst[0].x, pst[0].y, pst[0].z, pst[0].w, pst[1].x, pst[1].y, pst[1].z, pst[1].w};
      const float vv[8] = {pst[2].x, pst[2].y, pst[2].z, pst[2].w, pst[3].x, pst[3].y, pst[3].z, pst[3].w};
      const float gv[8] = {pst[4].x, pst[4].y, pst[4].z, pst[4].w, pst[5].x, pst[5].y, pst[5].z, pst[5].w};
      const float bv[8] = {pst[6].x, pst[6].y, pst[6].z, pst[6].w, pst[7].x, pst[7].y, pst[7].z, pst[7].w};
      float sc[8], sh[8];
      float plo, phi;
      act_clamp_bounds(pro.act, plo, phi);
#pragma unroll
      for (int k = 0; k < 8; ++k) {   // same arithmetic as bn.hip scale_shift8
        float mean = mv[k], var = vv[k];
        if (pbase) {
          mean = mv[k] * pro.inv_count;
          var = fmaxf(vv[k] * pro.inv_count - mean * mean, 0.f);
        }
        sc[k] = gv[k] * rsqrtf(var + pro.eps);
        sh[k] = bv[k] - mean * sc[k];
      }
      const bool hres = pro.res != nullptr;   // kernel-uniform
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        const bf16x8 y = __builtin_bit_cast(bf16x8, ra[i]);
        const bf16x8 rv = __builtin_bit_cast(bf16x8, hres ? prs[i] : u32x4{0u, 0u, 0u, 0u});
        bf16x8 o;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          // branch-free activation: clamp to the act's bounds (identity for none)
          o[k] = f2bf(fminf(fmaxf(bf2f(y[k]) * sc[k] + sh[k] + bf2f(rv[k]), plo), phi));
        }
        const u32x4 t = __builtin_bit_cast(u32x4, o);
        ra[i] = ((pz >> i) & 1) ? u32x4{0u, 0u, 0u, 0u} : t;
        if (pko[i] >= 0) *(u32x4*)(pro.keep + pko[i]) = ra[i];
      }
    }
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int row = (tid >> 3) + 32 * i;
      *(u32x4*)(a + row * BK + swz(row, cc) * 8) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int row = (tid >> 3) + 32 * i;
      *(u32x4*)(b + row * BK + swz(row, cc) * 8) = rb[i];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (kt0 < kt1 && PF == 2) {
    // two stages in flight in registers (the train-batch dgrad is latency-bound: a 64-deep
    // stage is a few MFMAs per wave against a memory round trip); unrolled by two so each
    // register set is named statically, every trip issues the same loads (counted vmcnt exact)
    u32x4 ra0[AR], rb0[BR], ra1[AR], rb1[BR];
    load_stage(kt0, ra0, rb0);
    store_stage(0, ra0, rb0);
    load_stage(kt0 + 1, ra1, rb1);
    __syncthreads();
    for (int kt = kt0; kt < kt1; kt += 2) {
      load_stage(kt + 2, ra0, rb0);      // LDS 0 holds stage kt, ra1 stage kt + 1
      mma_stage<BM, BN>(sA, sA + BM * BK, acc, lane, wm, wn);
      if (kt + 1 >= kt1) break;
      store_stage(1, ra1, rb1);
      __syncthreads();
      load_stage(kt + 3, ra1, rb1);      // LDS 1 holds stage kt + 1, ra0 stage kt + 2
      const bf16* a1 = sA + Smem<BM, BN>::STAGE;
      mma_stage<BM, BN>(a1, a1 + BM * BK, acc, lane, wm, wn);
      if (kt + 2 >= kt1) break;
      store_stage(0, ra0, rb0);
      __syncthreads();
    }
    __syncthreads();                     // the epilogue may reuse the stage LDS
  } else if (kt0 < kt1) {
    u32x4 ra[AR], rb[BR];
    load_stage(kt0, ra, rb);
    store_stage(0, ra, rb);
    __syncthreads();
    MA_STAMP(1);
#ifdef MERCURY_STAMPS
    unsigned long long lap[4] = {0, 0, 0, 0};
    unsigned long long tl = __builtin_amdgcn_s_memtime();
#endif
    int buf = 0;
    for (int kt = kt0; kt < kt1; ++kt) {
      const bool more = kt + 1 < kt1;
      if (more) load_stage(kt + 1, ra, rb);
      MA_LAP(0, tl);
      const bf16* a = sA + buf * Smem<BM, BN>::STAGE;
      mma_stage<BM, BN>(a, a + BM * BK, acc, lane, wm, wn);
      MA_LAP(1, tl);
      if (more) store_stage(buf ^ 1, ra, rb);
      MA_LAP(2, tl);
      __syncthreads();
      MA_LAP(3, tl);
      buf ^= 1;
    }
#ifdef MERCURY_STAMPS
    if (threadIdx.x == 0) {
      const int b_ = blockIdx.x + blockIdx.y * gridDim.x;
      if (b_ < 8192)
        for (int q = 0; q < 4; ++q) g_stamps[b_][4 + q] = lap[q];
    }
#endif
  }
  MA_STAMP(2);
  finish<BM, BN>(acc, smem, e, g.M, g.Ncols, m0, n0, bx, by, gx, gy);
  MA_STAMP(3);
}


// two register-staged stages in flight where the second register set fits (64-wide tiles)
template <int BM, int BN>
constexpr int PAIR_PF() { return BM * BN <= 64 * 128 ? 2 : 1; }

template <int BM, int BN, bool TRANS, int PF = 1>
__global__ __launch_bounds__(NT, (nt_occ<BM, BN>())) void igemm_nt_kernel(const bf16* __restrict__ src,
                                                          const bf16* __restrict__ wt,
                                                          ConvGeom g, EpiParams e,
                                                          int ktiles_per_split) {
  __shared__ __attribute__((aligned(16))) char smem[Smem<BM, BN>::bytes(2)];
  const ProParams none{};
  const int bx = gridDim.y == 1 ? xcd_tile(blockIdx.x, gridDim.x) : blockIdx.x;
  igemm_nt_body<BM, BN, TRANS, false, PF>(src, wt, g, e, ktiles_per_split, smem, bx, blockIdx.y,
                                          gridDim.x, gridDim.y, none);
}

// forward conv with the BN-apply prologue on its input (ProParams)
template <int BM, int BN>
__global__ __launch_bounds__(NT, (nt_occ<BM, BN>())) void igemm_pro_kernel(const bf16* __restrict__ src,
                                                           const bf16* __restrict__ wt,
                                                           ConvGeom g, EpiParams e,
                                                           int ktiles_per_split, ProParams pro) {
  __shared__ __attribute__((aligned(16))) char smem[Smem<BM, BN>::bytes(2)];
  const int bx = gridDim.y == 1 ? xcd_tile(blockIdx.x, gridDim.x) : blockIdx.x;
  igemm_nt_body<BM, BN, false, true>(src, wt, g, e, ktiles_per_split, smem, bx,
                                     blockIdx.y, gridDim.x, gridDim.y, pro);
}

template <int BM, int BN, bool TRANS>
void launch_main(const bf16* src, const bf16* wt, const ConvGeom& g, const EpiParams& e, int per,
                 dim3 grid, hipStream_t st) {
  // a grid that does not fill the chip twice over is latency-bound (the train batch): two
  // stages in flight per block where the second register set fits
  if constexpr (PAIR_PF<BM, BN>() == 2) {
#ifndef MERCURY_FWD_PF1   // (A/B builds: bench/build_variant.py with this flag)
    if (grid.x * grid.y <= 512) {
      hipLaunchKernelGGL((igemm_nt_kernel<BM, BN, TRANS, 2>), grid, dim3(NT), 0, st, src, wt, g, e,
                         per);
      return;
    }
#endif
  }
  hipLaunchKernelGGL((igemm_nt_kernel<BM, BN, TRANS>), grid, dim3(NT), 0, st, src, wt, g, e, per);
}

// split-K decomposition (clamped; no split when the tile counters would not fit)
inline void ig_grid(const ConvGeom& g, int BM, int BN, int splits, int& gx, int& per, int& gy) {
  const int mtiles = (g.M + BM - 1) / BM, ntiles = (g.Ncols + BN - 1) / BN;
  const int ktiles = (g.Kc + 7) / 8;
  splits = splits < 1 ? 1 : (splits > ktiles ? ktiles : splits);
  per = (ktiles + splits - 1) / splits;
  gy = (ktiles + per - 1) / per;
  gx = mtiles * ntiles;
  if (gx > SEM_INTS) gy = 1, per = ktiles;
}

template <int BM, int BN, bool TRANS>
void launch_cfg(const bf16* src, const bf16* wt, const ConvGeom& g, EpiParams e, int splits,
                hipStream_t st, const ProParams* pro) {
  int gx, per, gy;
  ig_grid(g, BM, BN, splits, gx, per, gy);
  if (gy == 1) e.slab = nullptr;
  if (pro != nullptr && !TRANS) {
    hipLaunchKernelGGL((igemm_pro_kernel<BM, BN>), dim3(gx, gy), dim3(NT), 0, st, src, wt, g, e,
                       per, *pro);
    return;
  }
  launch_main<BM, BN, TRANS>(src, wt, g, e, per, dim3(gx, gy), st);
}

// ---------------------------------------------------------------- two forward convs, one launch
// A downsampling block's first conv (3x3, stride 2) and its 1x1 shortcut conv read the same
// input and are independent: at the train batch each alone fills a fraction of the chip (the
// shortcut 7-8 us on its own), so one launch runs both -- blocks [0, A.gx * A.gy) are the first
// conv's (tile, K split), the rest the shortcut's.  Same tile shape for both (one template);
// each problem keeps its own epilogue (statistics, split-K slab).
struct IgProb {
  const bf16* src;
  const bf16* wt;
  ConvGeom g;
  EpiParams e;
  int per, gx, gy;
};

template <int BM, int BN, int PF>
__global__ __launch_bounds__(NT, (nt_occ<BM, BN>())) void igemm_dual_kernel(IgProb A, IgProb B) {
  __shared__ __attribute__((aligned(16))) char smem[Smem<BM, BN>::bytes(2)];
  const ProParams none{};
  int b = blockIdx.x;
  const bool first = b < A.gx * A.gy;              // block-uniform
  if (!first) b -= A.gx * A.gy;
  const IgProb& p = first ? A : B;
  const int bx0 = b % p.gx, by = b / p.gx;
  const int bx = p.gy == 1 ? xcd_tile(bx0, p.gx) : bx0;
  igemm_nt_body<BM, BN, false, false, PF>(p.src, p.wt, p.g, p.e, p.per, smem, bx, by, p.gx, p.gy,
                                          none);
}

template <int BM, int BN>
void dual_cfg(IgProb A, IgProb B, hipStream_t st) {
  const int grid = A.gx * A.gy + B.gx * B.gy;
  if constexpr (PAIR_PF<BM, BN>() == 2) {
    if (grid <= 512) {   // the latency-bound rule of launch_main
      hipLaunchKernelGGL((igemm_dual_kernel<BM, BN, 2>), dim3(grid), dim3(NT), 0, st, A, B);
      return;
    }
  }
  hipLaunchKernelGGL((igemm_dual_kernel<BM, BN, 1>), dim3(grid), dim3(NT), 0, st, A, B);
}

// ---------------------------------------------------------------- stride-2 dgrad classes
// A stride-2 dgrad as a TRANS gather evaluates all R*S taps for every input pixel although only
// the taps whose parity matches the pixel's reach it (3x3 pad 1: 1, 2, 2 or 4 of 9; 1x1: 1 or
// 0 of 1) -- 3/4 of its MFMAs multiply the zero page.  Split the input pixels into the four
// parity classes (h % 2, w % 2): class (ph, pw) is a stride-1 FORWARD gather of dy over
// (N, ceil-half H, ceil-half W) rows with only its own taps, and its output rows scatter to
// (n, 2i + ph, 2j + pw) (EpiParams rm_*).  The four classes run as one launch; a class with
// no taps (1x1: all but (0, 0)) writes zeros.
struct S2Geom {
  ConvGeom g[4];
  int pre[5];          // tile prefix over the classes
  int hc[4], wc[4];    // class row-space dims
  int H, W;            // dx spatial dims
};

template <int BM, int BN, int PF>
__global__ __launch_bounds__(NT, (nt_occ<BM, BN>())) void dgrad_s2_kernel(const bf16* __restrict__ dy,
                                                           const bf16* __restrict__ wt,
                                                           S2Geom sg, EpiParams e) {
  __shared__ __attribute__((aligned(16))) char smem[Smem<BM, BN>::bytes(2)];
  const int b = blockIdx.x;
  const int c = (b >= sg.pre[1]) + (b >= sg.pre[2]) + (b >= sg.pre[3]);   // uniform
  EpiParams ec = e;
  ec.rm_hc = sg.hc[c];
  ec.rm_wc = sg.wc[c];
  ec.rm_h = sg.H;
  ec.rm_w = sg.W;
  ec.rm_ph = c >> 1;
  ec.rm_pw = c & 1;
  const ProParams none{};
  const int bx = b - sg.pre[c];
  igemm_nt_body<BM, BN, false, false, PF>(dy, wt, sg.g[c], ec, 1 << 20, smem, bx, 0,
                                          sg.pre[c + 1] - sg.pre[c], 1, none);
}

template <int BM, int BN>
void s2_cfg(const bf16* dy, const bf16* wt, const S2Geom& sg, const EpiParams& e, hipStream_t st) {
  const int grid = sg.pre[4];
  if (grid == 0) return;
  if constexpr (PAIR_PF<BM, BN>() == 2) {
    if (grid <= 512) {
      hipLaunchKernelGGL((dgrad_s2_kernel<BM, BN, 2>), dim3(grid), dim3(NT), 0, st, dy, wt, sg, e);
      return;
    }
  }
  hipLaunchKernelGGL((dgrad_s2_kernel<BM, BN, 1>), dim3(grid), dim3(NT), 0, st, dy, wt, sg, e);
}

// ---------------------------------------------------------------- dgrad + wgrad pair launch
// The two backward GEMMs of a conv read the same dy and are independent; at small batch each
// alone leaves most of the 256 CUs idle, and a second stream costs a cross-queue graph edge per
// layer.  One launch runs both: blocks [0, nw) are weight-gradient tiles (the longer reduction
// goes first), the rest data-gradient tiles, in one LDS allocation sized for the larger body.
template <int DBM, int DBN, int WBM, int WBN>
__global__ __launch_bounds__(NT, 2) void bwd_pair_kernel(const bf16* __restrict__ dy,
                                                          const bf16* __restrict__ wt, ConvGeom g,
                                                          EpiParams e, int dper, int dgx, int dgy,
                                                          const bf16* __restrict__ x,
                                                          WgradGeom wg, float* __restrict__ dw,
                                                          int wper, int wgx, int wgy) {
  constexpr int DB = Smem<DBM, DBN>::bytes(2), WB = wgb::WgSmem<WBM, WBN>::BYTES;
  __shared__ __attribute__((aligned(16))) char smem[DB > WB ? DB : WB];
  const int nw = wgx * wgy;
  const int b = blockIdx.x;
  if (b < nw) {
    wgb::wgrad_body<WBM, WBN>(dy, x, wg, dw, wper, (bf16*)smem, b % wgx, b / wgx, wgy);
  } else {
    const int d = b - nw;
    const ProParams none{};
    // (no XCD renumbering here: measured +1 % step time -- the pair's wgrad blocks come first,
    // so the dgrad tiles' XCD placement is already rotated and interleaved with them)
    igemm_nt_body<DBM, DBN, true, false, PAIR_PF<DBM, DBN>()>(dy, wt, g, e, dper, smem, d % dgx,
                                                               d / dgx, dgx, dgy, none);
  }
}

// the same pair with a stride-2 dgrad as parity classes (S2Geom): blocks [0, nw) wgrad tiles,
// the rest class-dgrad tiles
template <int DBM, int DBN, int WBM, int WBN>
__global__ __launch_bounds__(NT, 2) void bwd_pair_s2_kernel(const bf16* __restrict__ dy,
                                                             const bf16* __restrict__ wt,
                                                             S2Geom sg, EpiParams e,
                                                             const bf16* __restrict__ x,
                                                             WgradGeom wg, float* __restrict__ dw,
                                                             int wper, int wgx, int wgy) {
  constexpr int DB = Smem<DBM, DBN>::bytes(2), WB = wgb::WgSmem<WBM, WBN>::BYTES;
  __shared__ __attribute__((aligned(16))) char smem[DB > WB ? DB : WB];
  const int nw = wgx * wgy;
  const int b = blockIdx.x;
  if (b < nw) {
    wgb::wgrad_body<WBM, WBN>(dy, x, wg, dw, wper, (bf16*)smem, b % wgx, b / wgx, wgy);
    return;
  }
  const int d = b - nw;
  const int c = (d >= sg.pre[1]) + (d >= sg.pre[2]) + (d >= sg.pre[3]);
  EpiParams ec = e;
  ec.rm_hc = sg.hc[c];
  ec.rm_wc = sg.wc[c];
  ec.rm_h = sg.H;
  ec.rm_w = sg.W;
  ec.rm_ph = c >> 1;
  ec.rm_pw = c & 1;
  const ProParams none{};
  igemm_nt_body<DBM, DBN, false, false, PAIR_PF<DBM, DBN>()>(
      dy, wt, sg.g[c], ec, 1 << 20, smem, d - sg.pre[c], 0, sg.pre[c + 1] - sg.pre[c], 1, none);
}

// A downsampling block's shortcut backward (1x1 stride 2: class dgrad + wgrad) and the block's
// last conv's backward (3x3 stride 1: dgrad + wgrad) both start from the block-final BN's
// backward and are independent: one launch runs the two pairs -- blocks [0, nA) the stride-1
// pair's wgrad then dgrad tiles, the rest the shortcut's wgrad then parity-class dgrad tiles
// (64 x 64 class tiles, 64 x 64 wgrad tiles: the train-batch shortcut plans).
struct PairProb {
  const bf16* dy;
  const bf16* wt;
  ConvGeom g;
  EpiParams e;
  int dper, dgx, dgy;
  const bf16* x;
  WgradGeom wg;
  float* dw;
  int wper, wgx, wgy;
};
struct S2PairProb {
  const bf16* dy;
  const bf16* wt;
  S2Geom sg;
  EpiParams e;
  const bf16* x;
  WgradGeom wg;
  float* dw;
  int wper, wgx, wgy;
};

template <int DBM, int DBN, int WBM, int WBN>
__global__ __launch_bounds__(NT, 2) void bwd_pair_sc_kernel(PairProb A, S2PairProb B) {
  constexpr int DB = Smem<DBM, DBN>::bytes(2), WB = wgb::WgSmem<WBM, WBN>::BYTES;
  constexpr int SB = Smem<64, 64>::bytes(2), SWB = wgb::WgSmem<64, 64>::BYTES;
  constexpr int M1 = DB > WB ? DB : WB, M2 = SB > SWB ? SB : SWB;
  __shared__ __attribute__((aligned(16))) char smem[M1 > M2 ? M1 : M2];
  const ProParams none{};
  int b = blockIdx.x;
  const int nwA = A.wgx * A.wgy, nA = nwA + A.dgx * A.dgy;
  if (b < nA) {                                         // block-uniform
    if (b < nwA) {
      wgb::wgrad_body<WBM, WBN>(A.dy, A.x, A.wg, A.dw, A.wper, (bf16*)smem, b % A.wgx, b / A.wgx,
                                A.wgy);
    } else {
      const int d = b - nwA;
      igemm_nt_body<DBM, DBN, true, false, PAIR_PF<DBM, DBN>()>(A.dy, A.wt, A.g, A.e, A.dper, smem,
                                                                 d % A.dgx, d / A.dgx, A.dgx,
                                                                 A.dgy, none);
    }
    return;
  }
  b -= nA;
  const int nwB = B.wgx * B.wgy;
  if (b < nwB) {
    wgb::wgrad_body<64, 64>(B.dy, B.x, B.wg, B.dw, B.wper, (bf16*)smem, b % B.wgx, b / B.wgx, B.wgy);
    return;
  }
  const int d = b - nwB;
  const int c = (d >= B.sg.pre[1]) + (d >= B.sg.pre[2]) + (d >= B.sg.pre[3]);
  EpiParams ec = B.e;
  ec.rm_hc = B.sg.hc[c];
  ec.rm_wc = B.sg.wc[c];
  ec.rm_h = B.sg.H;
  ec.rm_w = B.sg.W;
  ec.rm_ph = c >> 1;
  ec.rm_pw = c & 1;
  igemm_nt_body<64, 64, false, false, PAIR_PF<64, 64>()>(B.dy, B.wt, B.sg.g[c], ec, 1 << 20, smem,
                                                         d - B.sg.pre[c], 0,
                                                         B.sg.pre[c + 1] - B.sg.pre[c], 1, none);
}

template <int DBM, int DBN, int WBM, int WBN>
void pair_cfg(const bf16* dy, const bf16* wt, const ConvGeom& g, EpiParams e, int splits,
              const bf16* x, WgradGeom wg, float* dw, int wsplits, hipStream_t st) {
  int dgx, dper, dgy, wgx, wper, wgy;
  ig_grid(g, DBM, DBN, splits, dgx, dper, dgy);
  if (dgy == 1) e.slab = nullptr;
  wgb::wg_grid(wg, WBM, WBN, wsplits, wgx, wper, wgy);
  if (wgx > wgb::WG_SEM_INTS) wg.slab = nullptr;
  hipLaunchKernelGGL((bwd_pair_kernel<DBM, DBN, WBM, WBN>), dim3(dgx * dgy + wgx * wgy), dim3(NT),
                     0, st, dy, wt, g, e, dper, dgx, dgy, x, wg, dw, wper, wgx, wgy);
}

}  // namespace

int igemm_read_stamps(unsigned long long* host, int n) {
#ifdef MERCURY_STAMPS
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 12 * n) ==
         hipSuccess;
#else
  (void)host;
  (void)n;
  return 0;
#endif
}


size_t igemm_slab_bytes(const ConvGeom& g, int bm, int bn, int splits) {
  const size_t mtiles = (g.M + bm - 1) / bm, ntiles = (g.Ncols + bn - 1) / bn;
  return SEM_INTS * 4 + (size_t)splits * mtiles * ntiles * bm * bn * 4;
}

const bf16* conv_zero_page();
static const bf16* zero_page() { return conv_zero_page(); }

const bf16* conv_zero_page() {
  static const bf16* zp = nullptr;
  if (!zp) {
    void* p = nullptr;
    (void)hipGetSymbolAddress(&p, HIP_SYMBOL(g_zero_page));
    zp = (const bf16*)p;
  }
  return zp;
}

void igemm_launch(const bf16* src, const bf16* wt, const ConvGeom& g_in, const EpiParams& e,
                  int bm, int bn, int splits, bool trans, hipStream_t st, const ProParams* pro) {
  ConvGeom g = g_in;
  g.zero = zero_page();
#define MA_CASE(BM_, BN_)                                                           \
  if (bm == BM_ && bn == BN_) {                                                     \
    if (trans) launch_cfg<BM_, BN_, true>(src, wt, g, e, splits, st, nullptr);       \
    else launch_cfg<BM_, BN_, false>(src, wt, g, e, splits, st, pro);                \
    return;                                                                         \
  }
  MA_CASE(128, 128)
  MA_CASE(128, 64)
  MA_CASE(64, 128)
  MA_CASE(64, 64)
  MA_CASE(256, 64)
  MA_CASE(256, 128)
#undef MA_CASE
}

// both forward, plain input, the same tile (bm, bn); returns 0 when there is no instantiation
int igemm_dual_launch(const bf16* srcA, const bf16* wtA, const ConvGeom& gA, const EpiParams& eA,
                      int splitsA, const bf16* srcB, const bf16* wtB, const ConvGeom& gB,
                      const EpiParams& eB, int splitsB, int bm, int bn, hipStream_t st) {
  IgProb A{srcA, wtA, gA, eA, 0, 0, 0}, B{srcB, wtB, gB, eB, 0, 0, 0};
  A.g.zero = B.g.zero = zero_page();
  ig_grid(A.g, bm, bn, splitsA, A.gx, A.per, A.gy);
  ig_grid(B.g, bm, bn, splitsB, B.gx, B.per, B.gy);
  if (A.gy == 1) A.e.slab = nullptr;
  if (B.gy == 1) B.e.slab = nullptr;
  if (A.gy > 1 && B.gy > 1 && A.e.slab == B.e.slab) return 0;   // one slab per split problem
#define MA_CASE(BM_, BN_)                 \
  if (bm == BM_ && bn == BN_) {           \
    dual_cfg<BM_, BN_>(A, B, st);         \
    return 1;                             \
  }
  MA_CASE(64, 128)
  MA_CASE(128, 128)
  MA_CASE(128, 64)
  MA_CASE(64, 64)
#undef MA_CASE
  return 0;
}

// the four class geometries of a stride-2 dgrad (false: the conv does not qualify)
static bool s2_geom(const ConvGeom& gt, int bm, int bn, int H, int W, int N, S2Geom& sg) {
  // gt: the TRANS geometry (SH, SW = dy spatial, SC = dy channels, R, S, stride, pad, Ncols = C)
  if (gt.stride != 2 || (gt.SC & 63) || gt.R != gt.S) return false;
  if (!((gt.R == 3 && gt.pad == 1) || (gt.R == 1 && gt.pad == 0))) return false;
  sg = S2Geom{};
  sg.H = H;
  sg.W = W;
  sg.pre[0] = 0;
  for (int c = 0; c < 4; ++c) {
    const int ph = c >> 1, pw = c & 1;
    // taps reaching parity ph: r == (ph + pad) mod 2; virtual tap r' = 0.. reads r = trb - 2 r'
    int rv = 0, trb = -1;
    for (int r = gt.R - 1; r >= 0; --r)
      if (((ph + gt.pad - r) & 1) == 0) {
        if (trb < 0) trb = r;
        ++rv;
      }
    int sv = 0, tsb = -1;
    for (int s = gt.S - 1; s >= 0; --s)
      if (((pw + gt.pad - s) & 1) == 0) {
        if (tsb < 0) tsb = s;
        ++sv;
      }
    // the first virtual tap reads dy pixel i + (ph + pad - trb) / 2: zero offset for the
    // supported shapes (3x3 pad 1, 1x1 pad 0), so the class gather is stride 1, pad 0
    if ((rv && ph + gt.pad - trb != 0) || (sv && pw + gt.pad - tsb != 0)) return false;
    const int hc = (H - ph + 1) / 2, wc = (W - pw + 1) / 2;
    ConvGeom g{};
    g.SH = gt.SH;
    g.SW = gt.SW;
    g.SC = gt.SC;
    g.RP = hc;
    g.RQ = wc;
    g.R = rv > 0 ? rv : 1;
    g.S = sv > 0 ? sv : 1;
    g.stride = 1;
    g.pad = 0;
    g.Kc = (rv * sv) * (gt.SC >> 3);    // 0: no tap reaches the class -> zeros
    g.Ncols = gt.Ncols;
    g.M = N * hc * wc;
    g.zero = zero_page();
    g.ldb = gt.R * gt.S * gt.SC;
    g.trb = trb < 0 ? 0 : trb;
    g.tsb = tsb < 0 ? 0 : tsb;
    g.tS = gt.S;
    sg.g[c] = g;
    sg.hc[c] = hc;
    sg.wc[c] = wc;
    sg.pre[c + 1] = sg.pre[c] + ((g.M + bm - 1) / bm) * ((g.Ncols + bn - 1) / bn);
  }
  return true;
}

int dgrad_s2_launch(const bf16* dy, const bf16* wt, const ConvGeom& gt, const EpiParams& e_in,
                    int bm, int bn, int H, int W, int N, hipStream_t st) {
  S2Geom sg;
  if (!s2_geom(gt, bm, bn, H, W, N, sg)) return 0;
  EpiParams e = e_in;
  e.slab = nullptr;                     // one K slice per tile
#define MA_CASE(BM_, BN_)                    \
  if (bm == BM_ && bn == BN_) {              \
    s2_cfg<BM_, BN_>(dy, wt, sg, e, st);     \
    return 1;                                \
  }
  MA_CASE(128, 128)
  MA_CASE(128, 64)
  MA_CASE(64, 128)
  MA_CASE(64, 64)
  MA_CASE(256, 64)
#undef MA_CASE
  return 0;
}

int conv_bwd_pair_s2_launch(const bf16* dy, const bf16* wt, const ConvGeom& gt,
                            const EpiParams& e_in, int bm, int bn, int H, int W, int N,
                            const bf16* x, const WgradGeom& wg_in, float* dw, int wbm, int wbn,
                            int wsplits, hipStream_t st) {
  S2Geom sg;
  if (!s2_geom(gt, bm, bn, H, W, N, sg)) return 0;
  EpiParams e = e_in;
  e.slab = nullptr;
  WgradGeom wg = wg_in;
  wg.zero = zero_page();
#define MA_W(DBM_, DBN_, WBM_, WBN_)                                                        \
  if (bm == DBM_ && bn == DBN_ && wbm == WBM_ && wbn == WBN_) {                            \
    int wgx, wper, wgy;                                                                    \
    wgb::wg_grid(wg, WBM_, WBN_, wsplits, wgx, wper, wgy);                                 \
    if (wgx > wgb::WG_SEM_INTS) wg.slab = nullptr;                                         \
    hipLaunchKernelGGL((bwd_pair_s2_kernel<DBM_, DBN_, WBM_, WBN_>),                        \
                       dim3(sg.pre[4] + wgx * wgy), dim3(NT), 0, st, dy, wt, sg, e, x, wg, dw, \
                       wper, wgx, wgy);                                                    \
    return 1;                                                                              \
  }
  MA_W(64, 64, 64, 64)
  MA_W(64, 64, 128, 128)
  MA_W(64, 64, 64, 128)
  MA_W(64, 64, 128, 64)
#undef MA_W
  return 0;
}

// the stride-1 pair (conv_bwd_pair_launch's arguments) and the shortcut's stride-2 pair
// (conv_bwd_pair_s2_launch's, 64 x 64 tiles) in one launch; 0: no instantiation / not a pair
int conv_bwd_pair_sc_launch(const bf16* dyA, const bf16* wtA, const ConvGeom& gA_in,
                            const EpiParams& eA_in, int bm, int bn, int splits, const bf16* xA,
                            const WgradGeom& wgA_in, float* dwA, int wbm, int wbn,
                            int wsplits, const bf16* dyB, const bf16* wtB, const ConvGeom& gtB,
                            const EpiParams& eB_in, int HB, int WB, int NB, const bf16* xB,
                            const WgradGeom& wgB_in, float* dwB, int wsplitsB,
                            hipStream_t st) {
  PairProb A;
  A.dy = dyA;
  A.wt = wtA;
  A.g = gA_in;
  A.g.zero = zero_page();
  A.e = eA_in;
  A.x = xA;
  A.wg = wgA_in;
  A.wg.zero = A.g.zero;
  A.dw = dwA;
  ig_grid(A.g, bm, bn, splits, A.dgx, A.dper, A.dgy);
  if (A.dgy == 1) A.e.slab = nullptr;
  wgb::wg_grid(A.wg, wbm, wbn, wsplits, A.wgx, A.wper, A.wgy);
  if (A.wgx > wgb::WG_SEM_INTS) A.wg.slab = nullptr;
  S2PairProb B;
  if (!s2_geom(gtB, 64, 64, HB, WB, NB, B.sg)) return 0;
  B.dy = dyB;
  B.wt = wtB;
  B.e = eB_in;
  B.e.slab = nullptr;
  B.x = xB;
  B.wg = wgB_in;
  B.wg.zero = A.g.zero;
  B.dw = dwB;
  wgb::wg_grid(B.wg, 64, 64, wsplitsB, B.wgx, B.wper, B.wgy);
  if (B.wgx > wgb::WG_SEM_INTS) B.wg.slab = nullptr;
  if (A.wg.slab != nullptr && A.wg.slab == B.wg.slab) return 0;
  const int grid = A.wgx * A.wgy + A.dgx * A.dgy + B.wgx * B.wgy + B.sg.pre[4];
#define MA_SC(DBM_, DBN_, WBM_, WBN_)                                                       \
  if (bm == DBM_ && bn == DBN_ && wbm == WBM_ && wbn == WBN_) {                             \
    hipLaunchKernelGGL((bwd_pair_sc_kernel<DBM_, DBN_, WBM_, WBN_>), dim3(grid), dim3(NT), 0, st, \
                       A, B);                                                                \
    return 1;                                                                                \
  }
  MA_SC(64, 64, 64, 64)
  MA_SC(64, 64, 128, 128)
#undef MA_SC
  return 0;
}

int conv_bwd_pair_launch(const bf16* dy, const bf16* wt, const ConvGeom& g_in, const EpiParams& e,
                         int bm, int bn, int splits, const bf16* x, const WgradGeom& wg_in,
                         float* dw, int wbm, int wbn, int wsplits, hipStream_t st) {
  ConvGeom g = g_in;
  g.zero = zero_page();
  WgradGeom wg = wg_in;
  wg.zero = g.zero;
#define MA_W(DBM_, DBN_, WBM_, WBN_)                                                   \
  if (wbm == WBM_ && wbn == WBN_) {                                                   \
    pair_cfg<DBM_, DBN_, WBM_, WBN_>(dy, wt, g, e, splits, x, wg, dw, wsplits, st);   \
    return 1;                                                                         \
  }
#define MA_D(DBM_, DBN_)                                                               \
  if (bm == DBM_ && bn == DBN_) {                                                     \
    MA_W(DBM_, DBN_, 128, 128)                                                        \
    MA_W(DBM_, DBN_, 128, 64)                                                         \
    MA_W(DBM_, DBN_, 64, 128)                                                         \
    MA_W(DBM_, DBN_, 64, 64)                                                          \
  }
  MA_D(128, 128)
  MA_D(128, 64)
  MA_D(64, 128)
  MA_D(64, 64)
  MA_D(256, 64)
#undef MA_D
#undef MA_W
  return 0;   // no instantiation: caller launches the two kernels separately
}
