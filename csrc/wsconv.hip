// Weight-stationary persistent halo convolution (gfx950): stride-1 3x3 convs with 64 or 128
// input channels -- ResNet-18's layer1 / layer2 convs (`pytorch_model.py:19-36`) at
// the scoring batch, where hconv_persist (hconv.hip) spent its time streaming the SAME weight
// tiles through an LDS ring every tap and synchronising its 8 waves on a barrier per tap.
//
// The whole weight slice a block needs lives in REGISTERS for the kernel's lifetime:
//   C = 64 : block tile 256 rows x 64 output channels, 4 waves as 2 (rows) x 2 (columns); each
//            wave holds its 32 columns x 9 taps x 64 channels = 144 VGPRs of bf16 weights;
//   C = 128: block tile 128 rows x 128 channels, 4 waves as 1 x 4; 16 columns per wave would
//            feed one MFMA per A fragment, so each wave holds 32 columns x 9 taps x 128 channels
//            (288 registers: one wave per SIMD, the unified VGPR/AGPR file).
// What streams is only the input halo (the tile's input rows + one above / below, all columns,
// every 64-channel plane), LDS-DMA'd (`buffer_load_dwordx4 ... lds`) into the other of two LDS
// buffers while the current tile computes.  Per tile there is ONE barrier (halo swap); the taps
// run back to back from registers and LDS with no synchronisation, and LDS carries only the A
// fragments: 64 KB per tap per CU against 512 MFMA cycles per SIMD.
//
// Epilogue straight from the accumulators (lane l: output pixel l & 15, four consecutive
// channels = 8 contiguous NHWC bytes, one buffer store each); ghost-BN statistics (sum, sum of
// squares per channel and group) kept as running per-lane sums over the block's CONTIGUOUS tile
// range and flushed (DPP row sums -> LDS -> one atomic pair per channel) only when the group
// changes.  The halo wait before the next tile counts the stores issued after the DMA, so
// nothing drains.
//
// Host contract (ops/hconv.py wsconv_*): 3x3, stride 1, pad 1, C in {64, 128}, K % BN == 0,
// M % BM == 0, statistics groups a multiple of BM, tile = whole output rows of one image or
// whole images, halo <= HRC pieces per wave per plane, no bias / accumulate / prologue.
#include "conv_epi.h"

namespace {

MA_DEV unsigned ws_lds(const void* p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) char*)p;
}
// 16 bytes per lane, buffer -> LDS (lane l lands at the wave-uniform LDS address + 16 l).  Inline
// asm: the compiler must not see the DMA (it would answer every LDS read with a full drain).
MA_DEV void ws_dma16(__amdgpu_buffer_rsrc_t r, unsigned off, unsigned lds) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
               ::"v"(off), "s"(r), "s"(lds) : "memory");
}
template <int N>
MA_DEV void ws_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
constexpr unsigned WS_OOB = 0x7ffffff0u;   // past every tensor: the DMA lands zeros

template <int CS>
struct WsCfg {
  // C = 64: 256 x 64 tiles, waves 2 x 2 (wave tile 128 x 32); C = 128: 64 x 128 tiles, waves
  // 1 x 4 (wave tile 64 x 32) -- every wave's tile is 32 columns wide (two MFMAs per A fragment)
  static constexpr int BM = CS == 1 ? 256 : 64;
  static constexpr int BN = CS == 1 ? 64 : 128;
  static constexpr int WM = CS == 1 ? 2 : 1;
  static constexpr int NW = 4;
  static constexpr int WN = NW / WM;
  static constexpr int TM = BM / (16 * WM);   // 8 / 4
  static constexpr int TN = BN / (16 * WN);   // 2
  static constexpr int PPX = 8 * NW;          // halo pixels per DMA round (8 per wave)
};

template <int CS, int HWP, int HRC, bool STATS>
__global__ __launch_bounds__(256, 1) void wsconv_kernel(const bf16* __restrict__ src,
                                                        const bf16* __restrict__ wt,
                                                        HconvGeom g, EpiParams e) {
  using Cf = WsCfg<CS>;
  constexpr int BM = Cf::BM, BN = Cf::BN, WM = Cf::WM, WN = Cf::WN, TM = Cf::TM, TN = Cf::TN;
  constexpr int PPX = Cf::PPX, T = 9;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const int wm = w / WN, wn = w % WN;
  const int C = CS * 64;
  const int PQ = g.P * g.Q;
  const int ntn = g.K / BN;
  const int mtiles = g.N * PQ / BM;
  // block -> (N tile, contiguous range of M tiles): the weights are per N tile
  const int G = gridDim.x, b = blockIdx.x;
  const int gpn = G / ntn;                                  // blocks per N tile (host: G % ntn == 0)
  const int nt = b % ntn, bi = b / ntn;
  const int mt0 = (int)((long long)mtiles * bi / gpn), mt1 = (int)((long long)mtiles * (bi + 1) / gpn);
  if (mt0 >= mt1) return;
  const int n0 = nt * BN;

  // ---- stationary weights: wreg[tap][plane][k-half][tn], lane l: output channel
  // n0 + wn*(BN/WN) + tn*16 + (l & 15), input channels plane*64 + (kk*4 + (l >> 4))*8 .. + 7
  bf16x8 wreg[T][CS][2][TN];
  {
    const int chunk_lo = lane >> 4;
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int n = n0 + wn * (BN / WN) + tn * 16 + (lane & 15);
      const bf16* wrow = wt + (size_t)n * T * C;
#pragma unroll
      for (int t = 0; t < T; ++t)
#pragma unroll
        for (int s = 0; s < CS; ++s)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk)
            wreg[t][s][kk][tn] = *(const bf16x8*)(wrow + t * C + s * 64 + (kk * 4 + chunk_lo) * 8);
    }
  }

  // ---- halo slots of this thread (tile-invariant part): pixel (tid >> 3) + PPX i of the halo
  // image [IMG][HT][HWP]; logical chunk lc of the pixel's 8 (swizzled: LDS chunk c ^ (p & 7))
  const int HR = (g.HPIX + PPX - 1) / PPX;
  const int HBYTES = HR * PPX * 128;                         // one 64-channel plane
  const int BUFB = CS * HBYTES;                              // one halo buffer (all planes)
  const int per_img = g.HT * HWP;
  const int lc = (lane & 7) ^ (lane >> 3);
  constexpr int HROW_NONE = 0x4000;
  int hbase[HRC], hrow[HRC];
#pragma unroll
  for (int i = 0; i < HRC; ++i) {
    hbase[i] = 0;
    hrow[i] = HROW_NONE;
    const int pix = (tid >> 3) + PPX * i;
    if (i < HR && pix < g.HPIX) {
      const int img = pix / per_img, rem = pix - img * per_img;
      const int hr = rem / HWP, col = rem - hr * HWP;
      const int ww = col - 1;                                // pad 1
      if (col < g.HWd && (unsigned)ww < (unsigned)g.W) {
        hbase[i] = (((img * g.H + hr) * g.W + ww) * C + lc * 8) * 2;
        hrow[i] = hr;
      }
    }
  }
  unsigned hoff[HRC];
  const auto rs_src = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0,
                                                        (int)((size_t)g.N * g.H * g.W * C * 2),
                                                        0x00020000);
  const float rpq = 1.f / (float)PQ, rq = 1.f / (float)g.Q;
  auto set_halo = [&](int m0) {
    const int n0i = udiv24(m0, PQ, rpq);
    const int p0 = udiv24(m0 - n0i * PQ, g.Q, rq);
    const int h0 = p0 - 1;                                   // first halo input row (pad 1)
    const int toff = (n0i * g.H + h0) * g.W * C * 2;
#pragma unroll
    for (int i = 0; i < HRC; ++i)
      hoff[i] = (unsigned)(h0 + hrow[i]) < (unsigned)g.H ? (unsigned)(hbase[i] + toff) : WS_OOB;
  };
  const unsigned s_halo = ws_lds(smem);
  const unsigned s_dump = s_halo + 2 * BUFB + wu * 1024;
  auto issue_halo = [&](int buf) {
    int hr = HR;
    asm volatile("" : "+s"(hr));
#pragma unroll
    for (int s = 0; s < CS; ++s)
#pragma unroll
      for (int i = 0; i < HRC; ++i)
        ws_dma16(rs_src, hoff[i] + s * 128,
                 i < hr ? s_halo + buf * BUFB + s * HBYTES + (PPX * i + 8 * wu) * 128 : s_dump);
  };

  // ---- A-fragment LDS pixel of tap (0, 0) per fragment row block (tile-invariant).  HWP is a
  // multiple of 8 (host), so a tap row step r * HWP keeps every pixel's swizzle (p & 7): the
  // byte address of (tap (r, s), plane, k-half kk, fragment tm) is
  //   abuf[plane][s][tm] ^ (64 kk)  +  r * HWP * 128  (an immediate offset of the LDS read)
  int apix[TM];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int row = wm * (BM / WM) + tm * 16 + (lane & 15);
    const int img = row / (g.TR * g.Q), rem = row - img * g.TR * g.Q;
    const int tr = rem / g.Q, q = rem - tr * g.Q;
    apix[tm] = img * per_img + tr * HWP + q;
  }
  const int c16 = (lane >> 4);                               // logical chunk of the k = 0..31 half
  int abuf[CS][3][TM];
  auto set_abuf = [&](int buf) {
#pragma unroll
    for (int pl = 0; pl < CS; ++pl)
#pragma unroll
      for (int sc = 0; sc < 3; ++sc)
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
          const int p = apix[tm] + sc;
          abuf[pl][sc][tm] = buf * BUFB + pl * HBYTES + ((p << 3) + (c16 ^ (p & 7))) * 16;
        }
  };

  // ---- statistics: running per-lane sums over consecutive tiles of one group
  float* red = (float*)(smem + 2 * BUFB + Cf::NW * 1024);   // [WM][2][BN]
  float rs[TN][4], rss[TN][4];
#pragma unroll
  for (int tn = 0; tn < TN; ++tn)
#pragma unroll
    for (int j = 0; j < 4; ++j) rs[tn][j] = rss[tn][j] = 0.f;
  auto flush = [&](int grp) {
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        rs[tn][j] = row16_sum(rs[tn][j]);
        rss[tn][j] = row16_sum(rss[tn][j]);
      }
      if ((lane & 15) == 0) {
        const int cl = wn * (BN / WN) + tn * 16 + 4 * (lane >> 4);
        *(f32x4*)(red + (wm * 2) * BN + cl) = f32x4{rs[tn][0], rs[tn][1], rs[tn][2], rs[tn][3]};
        *(f32x4*)(red + (wm * 2 + 1) * BN + cl) = f32x4{rss[tn][0], rss[tn][1], rss[tn][2], rss[tn][3]};
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) rs[tn][j] = rss[tn][j] = 0.f;
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (tid < BN) {
      float a = 0.f, c = 0.f;
#pragma unroll
      for (int q = 0; q < WM; ++q) {
        a += red[(q * 2) * BN + tid];
        c += red[(q * 2 + 1) * BN + tid];
      }
      float* dst = e.stats + (size_t)grp * 2 * e.stats_ld + n0 + tid;
      atomicAdd(dst, a);
      atomicAdd(dst + e.stats_ld, c);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  };
  const auto rs_o = __builtin_amdgcn_make_buffer_rsrc((void*)e.out, 0,
                                                      (int)((size_t)g.N * PQ * e.ldo * 2),
                                                      0x00020000);
  typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));

  // ---- prologue: first halo, weights landed
  set_halo(mt0 * BM);
  issue_halo(0);
  ws_wait<0>();
  asm volatile("s_barrier" ::: "memory");
  int grp = STATS ? (mt0 * BM) / e.group_rows : 0;

  for (int mt = mt0; mt < mt1; ++mt) {
    const int buf = (mt - mt0) & 1;
    const bool more = mt + 1 < mt1;
    if (more) {
      set_halo((mt + 1) * BM);
      issue_halo(buf ^ 1);          // its last readers (tile mt - 1) passed the last barrier
    }
    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    set_abuf(buf);
    // steps (tap, plane, k-half) back to back; the fragments of step i + 1 are read while the
    // MFMAs of step i issue
    auto read = [&](bf16x8 (&fa)[TM], int t, int pl, int kk) {
      const int r = t / 3, sc = t % 3;
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
        fa[tm] = *(const bf16x8*)(smem + ((abuf[pl][sc][tm] ^ (kk * 64)) + r * HWP * 128));
    };
    constexpr int NSTEP = T * CS * 2;
    bf16x8 fa0[TM], fa1[TM];
    read(fa0, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);   // keep these reads out of the grouped region below
    // one step: its TM * TN MFMAs with the NEXT step's TM fragment reads interleaved (one read
    // per TN MFMAs, pinned by sched_group_barrier: left alone, hipcc re-serialises the reads
    // into one register quad with an lgkmcnt(0) before every pair of MFMAs)
    auto step = [&](bf16x8 (&cur)[TM], bf16x8 (&nxt)[TM], int st) {
      const int t = st / (2 * CS), pl = (st / 2) % CS, kk = st & 1;
      const int sn = st + 1;
      if (sn < NSTEP) read(nxt, sn / (2 * CS), (sn / 2) % CS, sn & 1);
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wreg[t][pl][kk][tn], cur[tm],
                                                               acc[tm][tn], 0, 0, 0);
      if (sn < NSTEP) {
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);    // DS read
          __builtin_amdgcn_sched_group_barrier(0x008, TN, 0);   // MFMA
        }
      }
    };
#pragma unroll
    for (int st = 0; st < NSTEP; st += 2) {
      step(fa0, fa1, st);
      step(fa1, fa0, st + 1);
    }
    // ---- epilogue: bf16 round, 8-byte stores from the accumulators, running statistics
    const int m0 = mt * BM;
    if (STATS) {
      const int g0 = m0 / e.group_rows;
      if (g0 != grp) {
        flush(grp);
        grp = g0;
      }
    }
    const int rbase = m0 + wm * (BM / WM) + (lane & 15);
    const int cbase = n0 + wn * (BN / WN) + 4 * (lane >> 4);
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        bf16x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = f2bf(acc[tm][tn][j]);
        const unsigned voff = (unsigned)(((rbase + tm * 16) * e.ldo + cbase + tn * 16) * 2);
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2v, o), rs_o, voff, 0, 0);
        if (STATS) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float f = bf2f(o[j]);
            rs[tn][j] += f;
            rss[tn][j] += f * f;
          }
        }
      }
    if (more) {
      // the next halo has landed (the TM*TN stores above are the only younger VMEM ops; a
      // flush's atomics only lengthen the wait) and every wave left this buffer
      ws_wait<TM * TN>();
      asm volatile("s_barrier" ::: "memory");
    }
  }
  if (STATS) flush(grp);
}

template <int CS, int HWP, int HRC>
int ws_launch_h(const bf16* src, const bf16* wt, const HconvGeom& g, const EpiParams& e, int grid,
                hipStream_t st) {
  using Cf = WsCfg<CS>;
  const int HR = (g.HPIX + Cf::PPX - 1) / Cf::PPX;
  const int bytes = 2 * CS * HR * Cf::PPX * 128 + Cf::NW * 1024 + Cf::WM * 2 * Cf::BN * 4;
  if (bytes > 160 * 1024) return 0;
  static bool attr[2] = {false, false};
  const bool stats = e.stats != nullptr;
  if (!attr[stats]) {
    (void)hipFuncSetAttribute(stats ? (const void*)wsconv_kernel<CS, HWP, HRC, true>
                                    : (const void*)wsconv_kernel<CS, HWP, HRC, false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr[stats] = true;
  }
  if (stats)
    hipLaunchKernelGGL((wsconv_kernel<CS, HWP, HRC, true>), dim3(grid), dim3(256), bytes, st, src,
                       wt, g, e);
  else
    hipLaunchKernelGGL((wsconv_kernel<CS, HWP, HRC, false>), dim3(grid), dim3(256), bytes, st, src,
                       wt, g, e);
  return 1;
}

// instantiated shapes: ResNet-18's stride-1 layer1 (32 x 32 x 64, halo pitch 40) and layer2
// (16 x 16 x 128, pitch 24)
int ws_dispatch(const bf16* src, const bf16* wt, const HconvGeom& g, const EpiParams& e, int grid,
                hipStream_t st) {
  const int CS = g.C / 64;
  const int hr = (g.HPIX + 31) / 32;
  if (CS == 1 && g.HWP == 40 && hr <= 16) return ws_launch_h<1, 40, 16>(src, wt, g, e, grid, st);
  if (CS == 2 && g.HWP == 24 && hr <= 8) return ws_launch_h<2, 24, 8>(src, wt, g, e, grid, st);
  return 0;
}

}  // namespace

// returns 0 when the conv is outside the kernel's contract (the caller keeps its other plan)
int wsconv_launch(const bf16* src, const bf16* wt, const HconvGeom& g, const EpiParams& e,
                  int grid, hipStream_t st) {
  if (g.R != 3 || g.stride != 1 || g.pad != 1 || g.HALF || g.HS != 1 || g.SR != 1) return 0;
  if (e.bias || e.accumulate || e.bw_sums || e.slab) return 0;
  const int CS = g.C / 64;
  if (g.C % 64 || (CS != 1 && CS != 2)) return 0;
  const int BM = CS == 1 ? WsCfg<1>::BM : WsCfg<2>::BM, BN = CS == 1 ? WsCfg<1>::BN : WsCfg<2>::BN;
  const int M = g.N * g.P * g.Q;
  if (M % BM || g.K % BN || g.IMG * g.TR * g.Q != BM) return 0;
  if (e.stats && e.group_rows % BM) return 0;
  const int ntn = g.K / BN;
  const int mtiles = M / BM;
  if (grid < ntn) grid = ntn;
  grid -= grid % ntn;
  if (grid > mtiles * ntn) grid = mtiles * ntn;
  return ws_dispatch(src, wt, g, e, grid, st);
}
