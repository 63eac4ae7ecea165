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
// Structure: 256 threads = 4 waves (2x2), BMxBN output tile, BK = 64 per stage,
// register-staged double-buffered LDS (global loads of stage t+1 are issued before
// the MFMAs of stage t and written to the other LDS buffer after them: one barrier
// per stage), XOR-swizzled LDS rows (16-B chunk c of row r lives at c ^ (r&7)) so
// the ds_read_b128 fragment reads are spread over the banks.  Split-K writes fp32
// partial tiles in MFMA fragment order (fully coalesced 16 B/lane) and a reducer
// with the same epilogue finishes them.
//
// Epilogue (fused): optional per-channel bias, bf16 rounding, per-(ghost-group,
// channel) BatchNorm sum/sum-of-squares from the rounded values (LDS pre-reduce,
// one atomic per column per block), optional accumulate-into-existing (dgrad of a
// residual), coalesced 16-B stores through an LDS-staged tile.
#include "common.h"
#include "igemm.h"

namespace {

constexpr int BK = 64;          // k elements per stage (8 chunks of 8)
constexpr int NT = 256;         // threads

MA_DEV int swz(int row, int chunk) { return chunk ^ (row & 7); }

template <int BM, int BN>
struct Smem {
  static constexpr int A_ELEMS = BM * BK;
  static constexpr int B_ELEMS = BN * BK;
  static constexpr int STAGE = A_ELEMS + B_ELEMS;
  static constexpr int LOOP_BYTES = 2 * STAGE * 2;
  static constexpr int EPI_BYTES = BM * (BN + 8) * 2 + 2 * BN * 4 * 2;
  static constexpr int BYTES = LOOP_BYTES > EPI_BYTES ? LOOP_BYTES : EPI_BYTES;
};

// ---------------------------------------------------------------- epilogue
// acc[tm][tn][j] holds OUT[row0 + tm*16 + (lane>>4)*4 + j][col0 + tn*16 + (lane&15)]
// with row0 = m0 + wm*(BM/2), col0 = n0 + wn*(BN/2).
template <int BM, int BN>
MA_DEV void epilogue_bf16(f32x4 (&acc)[BM / 32][BN / 32], char* smem, const EpiParams& e,
                          int M, int N, int m0, int n0) {
  constexpr int TM = BM / 32, TN = BN / 32, LDT = BN + 8;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  bf16* tile = (bf16*)smem;
  float* red = (float*)(smem + BM * LDT * 2);  // [2][BN] sum, sumsq
  const bool stats = e.stats != nullptr;
  if (stats) {
    for (int i = tid; i < 2 * BN; i += NT) red[i] = 0.f;
  }
  // bias loads hoisted and issued together (a conditional load per column would be
  // serialised behind its own vmcnt(0))
  float biasv[TN];
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) biasv[tn] = 0.f;
  if (e.bias) {
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int col = n0 + wn * (BN / 2) + tn * 16 + (lane & 15);
      biasv[tn] = e.bias[col < N ? col : N - 1];
    }
  }
  __syncthreads();
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) {
    const int cl = wn * (BN / 2) + tn * 16 + (lane & 15);
    const int col = n0 + cl;
    const float bias = biasv[tn];
    float s = 0.f, ss = 0.f;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int rl = wm * (BM / 2) + tm * 16 + (lane >> 4) * 4 + j;
        const bf16 v = f2bf(acc[tm][tn][j] + bias);
        tile[rl * LDT + cl] = v;
        if (stats && (m0 + rl) < M) {
          const float fv = bf2f(v);
          s += fv;
          ss += fv * fv;
        }
      }
    }
    if (stats) {
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      ss += __shfl_xor(ss, 16, 64);
      ss += __shfl_xor(ss, 32, 64);
      if (lane < 16) {
        atomicAdd(&red[cl], s);
        atomicAdd(&red[BN + cl], ss);
      }
    }
  }
  __syncthreads();
  if (stats) {
    const int g = m0 / e.group_rows;
    float* dst = e.stats + (size_t)g * 2 * e.stats_ld;
    for (int i = tid; i < BN; i += NT) {
      const int col = n0 + i;
      if (col < N) {
        atomicAdd(dst + col, red[i]);
        atomicAdd(dst + e.stats_ld + col, red[BN + i]);
      }
    }
  }
  // coalesced 16-byte stores
  constexpr int CPR = BN / 8;  // chunks per row
  for (int i = tid; i < BM * CPR; i += NT) {
    const int rl = i / CPR, ch = i - rl * CPR;
    const int row = m0 + rl, col = n0 + ch * 8;
    if (row >= M || col >= N) continue;
    bf16x8 v = *(const bf16x8*)(tile + rl * LDT + ch * 8);
    bf16* dst = e.out + (size_t)row * e.ldo + col;
    if (e.accumulate) {
      const bf16x8 o = *(const bf16x8*)dst;
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = f2bf(bf2f(v[k]) + bf2f(o[k]));
    }
    *(bf16x8*)dst = v;
  }
}

template <int BM, int BN, bool TRANS>
__global__ __launch_bounds__(NT, 2) void igemm_nt_kernel(const bf16* __restrict__ src,
                                                          const bf16* __restrict__ wt,
                                                          ConvGeom g, EpiParams e,
                                                          int ktiles_per_split) {
  constexpr int TM = BM / 32, TN = BN / 32;
  constexpr int AR = BM / 32, BR = BN / 32;  // rows per thread for A / B staging
  __shared__ __attribute__((aligned(16))) char smem[Smem<BM, BN>::BYTES];
  bf16* sA = (bf16*)smem;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int ntn = (g.Ncols + BN - 1) / BN;
  const int mt = blockIdx.x / ntn, nt = blockIdx.x - mt * ntn;
  const int m0 = mt * BM, n0 = nt * BN;
  const int ktiles = (g.Kc + 7) / 8;
  const int kt0 = blockIdx.y * ktiles_per_split;
  const int kt1 = min(ktiles, kt0 + ktiles_per_split);
  const int C8 = g.SC >> 3;
  const int Kelems = g.Kc * 8;

  // per-thread A rows: decode pixel once
  const int cc = tid & 7;
  int a_base[AR], a_h[AR], a_w[AR];
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    const int m = m0 + (tid >> 3) + 32 * i;
    if (m < g.M) {
      const int pq = g.RP * g.RQ;
      const int n = m / pq, rem = m - n * pq;
      const int p = rem / g.RQ, q = rem - p * g.RQ;
      a_base[i] = n * g.SH * g.SW;
      if (TRANS) {
        a_h[i] = p + g.pad;
        a_w[i] = q + g.pad;
      } else {
        a_h[i] = p * g.stride - g.pad;
        a_w[i] = q * g.stride - g.pad;
      }
    } else {
      a_base[i] = -1;
      a_h[i] = a_w[i] = 0;
    }
  }

  u32x4 ra[AR], rb[BR];
  // k-chunk -> (r, s, c8).  When C/8 is a multiple of 8 a whole 64-deep stage lies in one
  // filter tap, so (r, s, c8 base) advance incrementally without integer division.
  const bool fastk = (C8 & 7) == 0;
  int tr = 0, ts = 0, tc = 0;
  if (fastk) {
    const int k0c = kt0 * 8;
    const int rs = k0c / C8;
    tc = k0c - rs * C8;
    tr = rs / g.S;
    ts = rs - tr * g.S;
  }
  auto load_stage = [&](int kt) {
    const int kc = kt * 8 + cc;
    const bool kval = kc < g.Kc;
    int r = 0, s = 0, c8 = 0;
    if (fastk) {
      r = tr;
      s = ts;
      c8 = tc + cc;
      tc += 8;  // advance the stage cursor for the next call
      if (tc == C8) {
        tc = 0;
        if (++ts == g.S) {
          ts = 0;
          ++tr;
        }
      }
    } else if (kval) {
      const int rs = kc / C8;
      c8 = kc - rs * C8;
      r = rs / g.S;
      s = rs - r * g.S;
    }
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      u32x4 v = {0u, 0u, 0u, 0u};
      if (kval && a_base[i] >= 0) {
        int h, ww;
        bool ok;
        if (TRANS) {
          const int hp = a_h[i] - r, wp = a_w[i] - s;
          ok = hp >= 0 && wp >= 0;
          if (g.stride == 2) ok = ok && !((hp | wp) & 1);
          h = g.stride == 2 ? (hp >> 1) : hp;
          ww = g.stride == 2 ? (wp >> 1) : wp;
          ok = ok && h < g.SH && ww < g.SW;
        } else {
          h = a_h[i] + r;
          ww = a_w[i] + s;
          ok = h >= 0 && ww >= 0 && h < g.SH && ww < g.SW;
        }
        if (ok) v = *(const u32x4*)(src + (size_t)(a_base[i] + h * g.SW + ww) * g.SC + c8 * 8);
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int n = n0 + (tid >> 3) + 32 * i;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (kval && n < g.Ncols) v = *(const u32x4*)(wt + (size_t)n * Kelems + kc * 8);
      rb[i] = v;
    }
  };
  auto store_stage = [&](int buf) {
    bf16* a = sA + buf * Smem<BM, BN>::STAGE;
    bf16* b = a + Smem<BM, BN>::A_ELEMS;
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

  if (kt0 < kt1) {
    load_stage(kt0);
    store_stage(0);
    __syncthreads();
    int buf = 0;
    for (int kt = kt0; kt < kt1; ++kt) {
      const bool more = kt + 1 < kt1;
      if (more) load_stage(kt + 1);
      const bf16* a = sA + buf * Smem<BM, BN>::STAGE;
      const bf16* b = a + Smem<BM, BN>::A_ELEMS;
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
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
          for (int tn = 0; tn < TN; ++tn)
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[tm], fb[tn], acc[tm][tn], 0, 0, 0);
      }
      if (more) store_stage(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }

  if (e.slab) {
    // split-K partial in fragment order: [split][tile][TM*TN][256 threads] float4
    const size_t ntiles = (size_t)gridDim.x;
    f32x4* dst = (f32x4*)e.slab + ((size_t)blockIdx.y * ntiles + blockIdx.x) * (TM * TN) * NT;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) dst[(tm * TN + tn) * NT + tid] = acc[tm][tn];
    return;
  }
  epilogue_bf16<BM, BN>(acc, smem, e, g.M, g.Ncols, m0, n0);
}

template <int BM, int BN>
__global__ __launch_bounds__(NT) void splitk_reduce_kernel(ConvGeom g, EpiParams e, int splits) {
  constexpr int TM = BM / 32, TN = BN / 32;
  __shared__ __attribute__((aligned(16))) char smem[Smem<BM, BN>::EPI_BYTES];
  const int tid = threadIdx.x;
  const int ntn = (g.Ncols + BN - 1) / BN;
  const int mt = blockIdx.x / ntn, nt = blockIdx.x - mt * ntn;
  const size_t ntiles = gridDim.x;
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int sp = 0; sp < splits; ++sp) {
    const f32x4* src = (const f32x4*)e.slab + ((size_t)sp * ntiles + blockIdx.x) * (TM * TN) * NT;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) acc[tm][tn] += src[(tm * TN + tn) * NT + tid];
  }
  epilogue_bf16<BM, BN>(acc, smem, e, g.M, g.Ncols, mt * BM, nt * BN);
}

template <int BM, int BN, bool TRANS>
void launch_cfg(const bf16* src, const bf16* wt, const ConvGeom& g, EpiParams e, int splits,
                hipStream_t st) {
  const int mtiles = (g.M + BM - 1) / BM, ntiles = (g.Ncols + BN - 1) / BN;
  const int ktiles = (g.Kc + 7) / 8;
  splits = splits < 1 ? 1 : (splits > ktiles ? ktiles : splits);
  const int per = (ktiles + splits - 1) / splits;
  splits = (ktiles + per - 1) / per;
  dim3 grid(mtiles * ntiles, splits);
  if (splits == 1) {
    e.slab = nullptr;
    hipLaunchKernelGGL((igemm_nt_kernel<BM, BN, TRANS>), grid, dim3(NT), 0, st, src, wt, g, e, per);
  } else {
    EpiParams ep = e;  // the GEMM writes slabs; the reducer runs the real epilogue
    hipLaunchKernelGGL((igemm_nt_kernel<BM, BN, TRANS>), grid, dim3(NT), 0, st, src, wt, g, ep, per);
    hipLaunchKernelGGL((splitk_reduce_kernel<BM, BN>), dim3(mtiles * ntiles), dim3(NT), 0, st, g, e,
                       splits);
  }
}

}  // namespace

size_t igemm_slab_bytes(const ConvGeom& g, int bm, int bn, int splits) {
  const size_t mtiles = (g.M + bm - 1) / bm, ntiles = (g.Ncols + bn - 1) / bn;
  return (size_t)splits * mtiles * ntiles * bm * bn * 4;
}

void igemm_launch(const bf16* src, const bf16* wt, const ConvGeom& g, const EpiParams& e,
                  int bm, int bn, int splits, bool trans, hipStream_t st) {
#define MA_CASE(BM_, BN_)                                                \
  if (bm == BM_ && bn == BN_) {                                          \
    if (trans) launch_cfg<BM_, BN_, true>(src, wt, g, e, splits, st);    \
    else launch_cfg<BM_, BN_, false>(src, wt, g, e, splits, st);         \
    return;                                                              \
  }
  MA_CASE(128, 128)
  MA_CASE(128, 64)
  MA_CASE(64, 128)
  MA_CASE(64, 64)
  MA_CASE(256, 64)
#undef MA_CASE
}
