// Halo-tile implicit-GEMM convolution with the producer's BatchNorm fused into the operand
// staging (reference conv/BN/ReLU stack `pytorch_model.py:19-36,72-97`).
//
// Why a halo tile.  The generic implicit GEMM (igemm.hip) gathers every input pixel once per
// filter tap: a 3x3 conv moves 9x its input through each CU's vector-memory path, and on
// MI355X the per-CU load path -- not the MFMAs -- sets the pace of the register-staged loop
// (stamps: ~1.1k cycles of load issue per 64-deep stage against ~0.5k of MFMA).  Here a
// block's output tile is IMG whole images or TR whole output rows of one image, so the input
// it needs for one 64-channel slice is a small rectangle (the halo).  It is staged into LDS
// ONCE and every tap reads its A fragments from it at a uniform pixel offset; per stage only
// the BN x 64 weight tile streams in.
//
// Why the BN goes here.  A ResNet block's BatchNorm (+ residual, + shortcut BatchNorm) and
// ReLU are elementwise on the conv INPUT, and a halo stages each input element exactly once:
// applying scale/shift + activation there costs one FMA/max per element, not 9 (the reason the
// generic kernel's prologue was restricted to 1x1 convs).  The activation is also written back
// once (``keep``) where the training backward or the next residual needs it, by the blocks of
// the first N tile, for the pixels that tile owns.  So no standalone bn_apply pass remains in a
// ResNet forward except the last block's (read by the pooling head).
//
// Layout.  Halo pixel (img, hr, col) lives at LDS pixel index (img*HT + hr)*HWP + col, 128 B per
// pixel (the 64-channel slice), chunk c of pixel p at slot c ^ (p & 7).  Stride-2 3x3 convs
// store the even input columns first and the odd ones from HALF on, so consecutive output
// pixels read consecutive LDS pixels at every tap.  With the row pitch HWP chosen on the host
// by a model of ds_read_b128's lane groups (ops/hconv.py), every A-fragment read of the ResNet
// shapes is bank-conflict-free.  The weight tile uses the igemm.hip image ([row][64],
// chunk c ^ (row & 7)).  MFMA v_mfma_f32_16x16x32_bf16 with swapped operands (lane l: output
// pixel l&15, four consecutive channels), so the shared epilogue of conv_epi.h applies as is:
// ghost-BN statistics, split-K (over 64-channel slices) reduced in-launch by the last slice.
#include "conv_epi.h"

namespace {

MA_DEV int bswz(int row, int chunk) { return chunk ^ (row & 7); }

MA_DEV float act_f(float v, int act) {
  if (act == 1) return fmaxf(v, 0.f);
  if (act == 2) return fminf(fmaxf(v, 0.f), 6.f);
  return v;
}

// per-channel scale / shift of one BatchNorm for 8 channels (same arithmetic as bn.hip)
MA_DEV void bn_coef8(const float* stats, const float* rmean, const float* rvar, const float* gamma,
                     const float* beta, int C, int g, int ch, float inv_count, float eps,
                     float (&sc)[8], float (&sh)[8]) {
  float mean[8], var[8];
  if (stats) {
    const float* s = stats + (size_t)g * 2 * C + ch;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      mean[k] = s[k] * inv_count;
      var[k] = fmaxf(s[C + k] * inv_count - mean[k] * mean[k], 0.f);
    }
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      mean[k] = rmean[ch + k];
      var[k] = rvar[ch + k];
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sc[k] = gamma[ch + k] * rsqrtf(var[k] + eps);
    sh[k] = beta[ch + k] - mean[k] * sc[k];
  }
}

constexpr int HRMAX = 16;    // halo 16-B chunks per thread (HPIX * 8 <= 16 * 256)

template <int BM, int BN, int WM, int MODE>
__global__ __launch_bounds__(NT, 2) void hconv_kernel(const bf16* __restrict__ src,
                                                      const bf16* __restrict__ wt, HconvGeom g,
                                                      EpiParams e, HconvPro pro) {
  constexpr int WN = 4 / WM;
  constexpr int TM = BM / (16 * WM), TN = BN / (16 * WN);
  constexpr int BRW = BN / 32;                      // weight rows per thread per stage
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* halo = smem;
  bf16* sB = (bf16*)(smem + g.HPIX * 128);

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w / WN, wn = w % WN;
  const int ntn = (g.K + BN - 1) / BN;
  const int gx = gridDim.x, gy = gridDim.y;
  const int bx = gy == 1 ? xcd_tile(blockIdx.x, gx) : blockIdx.x;
  const int by = blockIdx.y;
  const int mt = bx / ntn, nt = bx - mt * ntn;
  const int m0 = mt * BM, n0 = nt * BN;
  const int PQ = g.P * g.Q;
  const int M = g.N * PQ;
  const int n0i = m0 / PQ;
  const int p0 = (m0 - n0i * PQ) / g.Q;
  const int cc = tid & 7;
  const int nchunks = g.C >> 6;
  const int cb0 = by * g.chunks_per_split;
  const int cb1 = min(nchunks, cb0 + g.chunks_per_split);
  const int T = g.R * g.R;
  const int Kt = T * g.C;
  const bf16* zp = g.zero;

  // ---- halo slots of this thread (the same for every 64-channel slice): source element
  // offset of channel chunk cc of slice 0 (or -1: padding / beyond the batch), and whether the
  // pixel belongs to this tile (activation write-back).  Slot i is halo pixel (tid >> 3) + 32 i,
  // so its LDS byte offset is hbase + 4096 i (pixel & 7 is the same for every i).
  const int HR = (g.HPIX * 8 + NT - 1) / NT;
  int hsrc[HRMAX];
  unsigned own = 0;
  const int per_img = g.HT * g.HWP;
  const int h0 = p0 * g.stride - g.pad;
  const int hbase = ((tid >> 3) * 8 + (cc ^ ((tid >> 3) & 7))) * 16;
#pragma unroll
  for (int i = 0; i < HRMAX; ++i) {
    hsrc[i] = -1;
    const int pix = (tid >> 3) + 32 * i;
    if (i < HR && pix < g.HPIX) {
      const int img = pix / per_img, rem = pix - img * per_img;
      const int hr = rem / g.HWP, col = rem - hr * g.HWP;
      int hc;
      bool ok;
      if (g.HALF) {
        hc = col < g.HALF ? 2 * col : 2 * (col - g.HALF) + 1;
        ok = col < g.HALF ? col < (g.HWd + 1) / 2 : col - g.HALF < g.HWd / 2;
      } else {
        hc = col;
        ok = col < g.HWd;
      }
      const int h = h0 + hr * g.HS, ww = hc * g.HS - g.pad, n = n0i + img;
      ok = ok && n < g.N && (unsigned)h < (unsigned)g.H && (unsigned)ww < (unsigned)g.W;
      if (ok) {
        hsrc[i] = ((n * g.H + h) * g.W + ww) * g.C + cc * 8;
        // the tile owns input rows [p0*stride, (p0+TR)*stride) of its images (all columns)
        if (h >= p0 * g.stride && h < (p0 + g.TR) * g.stride) own |= 1u << i;
      }
    }
  }
  const bool keep = MODE > 0 && pro.keep != nullptr && nt == 0;   // host: only when owned = all
  const int grp = MODE > 0 ? n0i / pro.group_imgs : 0;

  // ---- A-fragment rows of this lane: LDS pixel of tap (0, 0) for each fragment
  int apix[TM];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int row = wm * (BM / WM) + tm * 16 + (lane & 15);
    const int img = row / (g.TR * g.Q), rem = row - img * g.TR * g.Q;
    const int tr = rem / g.Q, q = rem - tr * g.Q;
    const int hc = q * g.SR;
    const int col = g.HALF ? ((hc & 1) * g.HALF + (hc >> 1)) : hc;
    apix[tm] = img * per_img + tr * g.SR * g.HWP + col;
  }
  int boff[BRW];
#pragma unroll
  for (int i = 0; i < BRW; ++i) {
    const int n = n0 + (tid >> 3) + 32 * i;
    boff[i] = n < g.K ? n * Kt : -1;
  }

  // ---- staging helpers
  auto stage_halo = [&](int cb) {
    // load, (MODE) normalise + residual + activation, write back the owned pixels, LDS store;
    // in batches so at most 8 (4 with a second input) 16-byte loads per thread are in flight
    constexpr int BATCH = MODE >= 2 ? 4 : 8;
    float sc[8], sh[8], sc2[8], sh2[8];
    if constexpr (MODE > 0) {
      const int ch = cb * 64 + cc * 8;
      bn_coef8(pro.stats, pro.rmean, pro.rvar, pro.gamma, pro.beta, g.C, grp, ch, pro.inv_count,
               pro.eps, sc, sh);
      if constexpr (MODE == 3)
        bn_coef8(pro.stats2, pro.rmean2, pro.rvar2, pro.gamma2, pro.beta2, g.C, grp, ch,
                 pro.inv_count, pro.eps, sc2, sh2);
    }
#pragma unroll
    for (int i0 = 0; i0 < HRMAX; i0 += BATCH) {
      if (i0 >= HR) break;
      u32x4 v[BATCH], r[BATCH];
#pragma unroll
      for (int j = 0; j < BATCH; ++j) {
        const int o = hsrc[i0 + j];
        v[j] = *(const u32x4*)(o >= 0 ? src + o + cb * 64 : zp);
        if constexpr (MODE == 2) r[j] = *(const u32x4*)(o >= 0 ? pro.res + o + cb * 64 : zp);
        if constexpr (MODE == 3) r[j] = *(const u32x4*)(o >= 0 ? pro.y2 + o + cb * 64 : zp);
      }
#pragma unroll
      for (int j = 0; j < BATCH; ++j) {
        const int i = i0 + j;
        if constexpr (MODE > 0) {
          const bf16x8 y = __builtin_bit_cast(bf16x8, v[j]);
          const bf16x8 rr = __builtin_bit_cast(bf16x8, r[j]);
          bf16x8 o;
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            float a = bf2f(y[k]) * sc[k] + sh[k];
            if constexpr (MODE == 2) a += bf2f(rr[k]);
            if constexpr (MODE == 3) a += bf2f(rr[k]) * sc2[k] + sh2[k];
            o[k] = f2bf(act_f(a, pro.act));
          }
          // padding stays zero in ACTIVATION space (the conv pads the normalised input)
          v[j] = hsrc[i] >= 0 ? __builtin_bit_cast(u32x4, o) : u32x4{0u, 0u, 0u, 0u};
          if (keep && ((own >> i) & 1)) *(u32x4*)(pro.keep + hsrc[i] + cb * 64) = v[j];
        }
        if (i < HR && (tid >> 3) + 32 * i < g.HPIX) *(u32x4*)(halo + hbase + 4096 * i) = v[j];
      }
    }
  };

  u32x4 rb[BRW];
  auto load_b = [&](int cb, int t) {
    const int k = t * g.C + cb * 64 + cc * 8;
#pragma unroll
    for (int i = 0; i < BRW; ++i) rb[i] = *(const u32x4*)(boff[i] >= 0 ? wt + boff[i] + k : zp);
  };
  auto store_b = [&](int buf) {
    bf16* b = sB + buf * (BN * BK);
#pragma unroll
    for (int i = 0; i < BRW; ++i) {
      const int row = (tid >> 3) + 32 * i;
      *(u32x4*)(b + row * BK + bswz(row, cc) * 8) = rb[i];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (cb0 < cb1) {
    const int nst = (cb1 - cb0) * T;
    load_b(cb0, 0);
    stage_halo(cb0);
    store_b(0);
    __syncthreads();
    for (int s = 0; s < nst; ++s) {
      const int cl = s / T, t = s - cl * T;
      const int cb = cb0 + cl;
      const bool more = s + 1 < nst;
      if (more) load_b(t + 1 < T ? cb : cb + 1, t + 1 < T ? t + 1 : 0);
      // A from the halo at the tap's uniform pixel offset, B from the weight stage
      const int r = t / g.R, ss = t - r * g.R;
      const int toff = g.HALF ? r * g.HWP + (ss >> 1) + (ss & 1) * g.HALF : r * g.HWP + ss;
      const bf16* b = sB + (s & 1) * (BN * BK);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int chunk = kk * 4 + (lane >> 4);
        bf16x8 fa[TM], fb[TN];
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
          const int p = apix[tm] + toff;
          fa[tm] = *(const bf16x8*)(halo + (p * 8 + (chunk ^ (p & 7))) * 16);
        }
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
          const int row = wn * (BN / WN) + tn * 16 + (lane & 15);
          fb[tn] = *(const bf16x8*)(b + row * BK + bswz(row, chunk) * 8);
        }
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
          for (int tn = 0; tn < TN; ++tn)
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[tn], fa[tm], acc[tm][tn], 0, 0, 0);
      }
      if (t == T - 1 && more) {
        __syncthreads();                 // every wave is done with this slice's halo
        stage_halo(cb + 1);
      }
      if (more) store_b((s + 1) & 1);
      __syncthreads();
    }
  }
  finish<BM, BN, WM>(acc, smem, e, M, g.K, m0, n0, bx, by, gx, gy);
}

template <int BM, int BN, int WM, int MODE>
void launch_one(const bf16* src, const bf16* wt, const HconvGeom& g, const EpiParams& e,
                const HconvPro& pro, dim3 grid, hipStream_t st) {
  const int main_bytes = g.HPIX * 128 + 2 * BN * BK * 2;
  const int red = Smem<BM, BN>::RED_BYTES;
  const int bytes = main_bytes > red ? main_bytes : red;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)hconv_kernel<BM, BN, WM, MODE>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL((hconv_kernel<BM, BN, WM, MODE>), grid, dim3(NT), bytes, st, src, wt, g, e,
                     pro);
}

template <int BM, int BN, int WM>
void launch_mode(const bf16* src, const bf16* wt, const HconvGeom& g, const EpiParams& e,
                 const HconvPro& pro, dim3 grid, hipStream_t st) {
  switch (pro.mode) {
    case 1: launch_one<BM, BN, WM, 1>(src, wt, g, e, pro, grid, st); break;
    case 2: launch_one<BM, BN, WM, 2>(src, wt, g, e, pro, grid, st); break;
    case 3: launch_one<BM, BN, WM, 3>(src, wt, g, e, pro, grid, st); break;
    default: launch_one<BM, BN, WM, 0>(src, wt, g, e, pro, grid, st); break;
  }
}

}  // namespace

int hconv_launch(const bf16* src, const bf16* wt, const HconvGeom& g_in, const EpiParams& e_in,
                 const HconvPro& pro, int bm, int bn, int splits, hipStream_t st) {
  HconvGeom g = g_in;
  g.zero = conv_zero_page();
  EpiParams e = e_in;
  const int M = g.N * g.P * g.Q;
  const int gx = ((M + bm - 1) / bm) * ((g.K + bn - 1) / bn);
  const int nchunks = g.C >> 6;
  splits = splits < 1 ? 1 : (splits > nchunks ? nchunks : splits);
  g.chunks_per_split = (nchunks + splits - 1) / splits;
  int gy = (nchunks + g.chunks_per_split - 1) / g.chunks_per_split;
  if (gx > 1024) gy = 1, g.chunks_per_split = nchunks;    // tile counters: SEM_INTS
  if (gy == 1) e.slab = nullptr;
  const dim3 grid(gx, gy);
#define HC_CASE(BM_, BN_, WM_)                                  \
  if (bm == BM_ && bn == BN_) {                                 \
    launch_mode<BM_, BN_, WM_>(src, wt, g, e, pro, grid, st);   \
    return 1;                                                   \
  }
  HC_CASE(256, 64, 4)
  HC_CASE(128, 64, 2)
  HC_CASE(64, 64, 1)
  HC_CASE(128, 128, 2)
  HC_CASE(64, 128, 1)
#undef HC_CASE
  return 0;
}
