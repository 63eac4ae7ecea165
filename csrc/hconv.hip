// Halo-tile implicit-GEMM convolution, the persistent variants with the producer's BatchNorm
// fused into the operand staging (reference conv/BN/ReLU stack
// `pytorch_model.py:19-36,72-97`).
//
// Why a halo tile.  The generic implicit GEMM (igemm.hip) gathers every input pixel once per
// filter tap: a 3x3 conv moves 9x its input through each CU's vector-memory path.  Here a
// block's output tile is IMG whole images or TR whole output rows of one image, so the input
// it needs for one 64-channel slice is a small rectangle (the halo), staged into LDS ONCE and
// read by every tap at a uniform pixel offset; per tap only the BN x 64 weight tile streams in.
//
// Why the BN goes here.  A ResNet block's intra-block BatchNorm and ReLU are elementwise on the
// conv INPUT, and a halo stages each input element exactly once: applying scale/shift +
// activation there costs one FMA/max per element, not 9 (the persistent kernels' MODE 1, the
// scoring pass; the per-tile kernel below runs plain input: its staged BN modes measured
// slower than a bn_apply pass, profiles/r2/ab_fuse_bn_halo.json, and were removed).
//
// Pipeline (everything global -> LDS is LDS-DMA, `global_load_lds_dwordx4`, so no VGPR ever
// holds a tile in flight and every wait is an explicit counted `s_waitcnt vmcnt`):
//   * weights: a 3-slot ring, the tile of step s + 2 issued while step s computes;
//   * halo: slice c + 1's raw halo is issued in pieces during taps 0..T-3 of slice c into the
//     second halo buffer (single-slice tiles use one buffer, two blocks share a CU instead);
//   * one barrier per step (a ring slot is rewritten only after every wave left it).
// Issue counts per step are uniform by construction (halo pieces past the last load the zero
// page into a dump area), so each wait is one of four immediates.
//
// Layout.  Halo pixel (img, hr, col) lives at LDS pixel index (img*HT + hr)*HWP + col, 128 B per
// pixel (the 64-channel slice), chunk c of pixel p at slot c ^ (p & 7).  Stride-2 3x3 convs
// store the even input columns first and the odd ones from HALF on, so consecutive output
// pixels read consecutive LDS pixels at every tap.  The row pitch HWP is chosen on the host by
// a model of ds_read_b128's lane groups (mercury_amd/ops/hconv.py) so every A-fragment read of
// the ResNet shapes is bank-conflict-free.  The weight slot uses the igemm.hip image ([row][64],
// chunk c ^ (row & 7)).  MFMA v_mfma_f32_16x16x32_bf16 with swapped operands (lane l: output
// pixel l&15, four consecutive channels), so the shared epilogue of conv_epi.h applies as is:
// ghost-BN statistics, split-K (over 64-channel slices) reduced in-launch by the last slice.
#include "conv_epi.h"

namespace {

constexpr int NSLOT = 3;     // weight ring slots (prefetch distance 2)
constexpr int HRMAX = 16;    // halo DMA pieces per wave (32 pixels per piece over 4 waves)

// Activation as one clamp [lo, hi] (none: NaN bounds = identity that keeps NaN, relu: 0..inf,
// relu6: 0..6; conv_epi.h act_clamp_bounds) -- branch-free: a per-element if-chain on the
// kernel-uniform selector compiled to two scalar branches per element (255 in one halo
// transform, ~3x the transform's cost)
MA_DEV void act_bounds(int act, float& lo, float& hi) { act_clamp_bounds(act, lo, hi); }

// 16 bytes per lane, global -> LDS (`global_load_lds_dwordx4`), lane l landing at the wave-uniform
// LDS address + 16 l.  Issued from inline asm on purpose: the compiler models LDS-DMA as an LDS
// event of unknown order and then answers every fragment read with lgkmcnt(0) (measured on the
// ROCm 7.2 hipcc), so it must not see these; their completion is tracked by our own vmcnt waits.
MA_DEV void dma16(const void* src, unsigned lds) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
               ::"v"(src), "s"(lds) : "memory", "m0");
}

MA_DEV unsigned lds_addr(const void* p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) char*)p;
}

// zero source for padding halo pixels: one 64-channel slice per possible slice offset
__device__ __attribute__((aligned(16))) bf16 g_hzero[64 * 17];

template <int N>
MA_DEV void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Workgroup barrier WITHOUT the release fence of __syncthreads (whose vmcnt(0) would drain the
// LDS-DMA ring every step).  DMA visibility comes from each wave's counted vmcnt before it;
// the memory clobber keeps the compiler from moving LDS accesses across it.
MA_DEV void bar_raw() { asm volatile("s_barrier" ::: "memory"); }
// ... after this wave's LDS writes have completed
MA_DEV void bar_lds() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int BM, int BN, int WM>
__global__ __launch_bounds__(NT, 1) void hconv_kernel(const bf16* __restrict__ src,
                                                      const bf16* __restrict__ wt, HconvGeom g,
                                                      EpiParams e) {
  constexpr int WN = 4 / WM;
  constexpr int TM = BM / (16 * WM), TN = BN / (16 * WN);
  constexpr int BI = BN / 32;                       // weight DMA pieces per wave per step
  constexpr int HI = 3;                             // halo pieces per wave per prefetch step
  constexpr int SLOT = BN * 128;                    // bytes per weight slot
  constexpr int R = 3, T = R * R;                   // 3x3 filters (1x1 convs stay on igemm)
  constexpr int HP = T - 2;                         // taps that carry next-slice halo pieces
  static_assert(T % NSLOT == 0, "ring slot = tap % NSLOT");
  extern __shared__ __attribute__((aligned(16))) char smem[];

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
  const int nchunks = g.C >> 6;
  const int cb0 = by * g.chunks_per_split;
  const int cb1 = min(nchunks, cb0 + g.chunks_per_split);
  const int nsl = cb1 - cb0;
  const int nst = nsl * T;
  const int Kt = T * g.C;
  const int HR = (g.HPIX + 31) >> 5;                // DMA pieces per wave for a whole halo
  const int HBYTES = HR * 32 * 128;
  const int NH = g.chunks_per_split > 1 ? 2 : 1;
  char* ring = smem + NH * HBYTES;
  const int lc = (lane & 7) ^ (lane >> 3);          // logical chunk this lane fetches

  // ---- halo slots of this thread: slot j is pixel (tid >> 3) + 32 j; source element offset
  // of its logical chunk lc in slice 0 (or -1: padding / beyond the batch)
  int hsrc[HRMAX];
  const bf16* hptr[HRMAX];                          // DMA source of slice 0 (zero rows for pads)
  const int per_img = g.HT * g.HWP;
  const int h0 = p0 * g.stride - g.pad;
#pragma unroll
  for (int i = 0; i < HRMAX; ++i) {
    hsrc[i] = -1;
    const int pix = (tid >> 3) + 32 * i;
    if (i < HR && pix < g.HPIX) {
      const int img = pix / per_img, rem = pix - img * per_img;
      const int hr = rem / g.HWP, col = rem - hr * g.HWP;
      // this lane's physical chunk (lane & 7) of pixel pix holds logical chunk
      // (lane & 7) ^ swz(pix), swz(p) = (p + SWA * halo_row(p)) & 7 (pix & 7 == lane >> 3)
      const int lcs = (lane & 7) ^ (((lane >> 3) + g.SWA * hr) & 7);
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
      if (ok) hsrc[i] = ((n * g.H + h) * g.W + ww) * g.C + lcs * 8;
    }
  }
#pragma unroll
  for (int i = 0; i < HRMAX; ++i) hptr[i] = hsrc[i] >= 0 ? src + hsrc[i] : g_hzero + lc * 8;

  // ---- A-fragment rows of this lane: LDS pixel of tap (0, 0) for each fragment
  int apix[TM], aswz[TM];                           // aswz: p + SWA * halo_row at tap (0, 0)
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int row = wm * (BM / WM) + tm * 16 + (lane & 15);
    const int img = row / (g.TR * g.Q), rem = row - img * g.TR * g.Q;
    const int tr = rem / g.Q, q = rem - tr * g.Q;
    const int hc = q * g.SR;
    const int col = g.HALF ? ((hc & 1) * g.HALF + (hc >> 1)) : hc;
    apix[tm] = img * per_img + tr * g.SR * g.HWP + col;
    aswz[tm] = apix[tm] + g.SWA * tr * g.SR;
  }
  // weight rows this lane fetches (DMA piece j covers rows 8 * (w + 4 j) .. + 8)
  // (the host guarantees K % BN == 0: every weight row exists)
  const bf16* bptr[BI];
#pragma unroll
  for (int j = 0; j < BI; ++j) {
    const int n = n0 + 8 * (w + 4 * j) + (lane >> 3);
    bptr[j] = wt + (size_t)n * Kt + lc * 8;
  }
  // wave-uniform LDS byte addresses (scalar: no per-DMA readfirstlane / pointer casts)
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const unsigned s_halo = lds_addr(smem);
  const unsigned s_ring = s_halo + NH * HBYTES;
  const unsigned s_dump = s_ring + NSLOT * SLOT + wu * 1024;

  // ---- issue helpers (wave-uniform LDS bases)
  // weight tile of (slice cb, tap t) into ring slot `slot`
  auto issue_b = [&](int cb, int t, int slot) {
    const int k = t * g.C + cb * 64;
#pragma unroll
    for (int j = 0; j < BI; ++j)
      dma16(bptr[j] + k, s_ring + slot * SLOT + 8 * (wu + 4 * j) * 128);
  };
  // halo DMA piece j (compile-time: the tap loop is unrolled) of slice cb into buffer buf.  A
  // piece past the halo's last loads zeros into a 4 KB dump area, so every prefetch tap issues
  // exactly HI pieces and the counted waits hold.
  auto issue_h = [&](int cb, int buf, int j) {
    const bool v = j < HR;
    dma16(hptr[j] + cb * 64, v ? s_halo + buf * HBYTES + (32 * j + 8 * wu) * 128 : s_dump);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  MA_STAMP(0);
#ifdef MERCURY_STAMPS
  unsigned long long lap[4] = {0, 0, 0, 0};
  unsigned long long tl = __builtin_amdgcn_s_memtime();
#endif
  if (nst > 0) {
    // prologue: the first slice's whole halo, then the weight tiles of steps 0 and 1
#pragma unroll
    for (int j = 0; j < HRMAX; ++j)
      if (j < HR) issue_h(cb0, 0, j);
    issue_b(cb0, 0, 0);
    issue_b(cb0, 1, 1);                           // nst >= T = 9
    for (int cl = 0; cl < nsl; ++cl) {
      const int buf = NH == 2 ? (cl & 1) : 0;
      const bool more = NH == 2 && cl + 1 < nsl;  // prefetch the next slice's halo
      // this slice's halo: everything but the two newest weight tiles has landed
      vm_wait<2 * BI>();
      bar_raw();
      if (cl == 0) MA_STAMP(1);
      MA_LAP(3, tl);
      const char* hb = smem + buf * HBYTES;
#pragma unroll
      for (int t = 0; t < T; ++t) {
        const int s = cl * T + t;
        // weight tile of step s: newer are the halo pieces of step s-1 and the tile of s+1
        const bool hprev = more && t >= 1 && t - 1 < HP;
        const bool nxt = s + 1 < nst;
        if (hprev) {
          if (nxt) vm_wait<HI + BI>();
          else vm_wait<HI>();
        } else {
          if (nxt) vm_wait<BI>();
          else vm_wait<0>();
        }
        bar_raw();
        MA_LAP(0, tl);
        if (more && t < HP) {
#pragma unroll
          for (int q = 0; q < HI; ++q) {
            const int j = t * HI + q;
            issue_h(cb0 + cl + 1, buf ^ 1, j < HRMAX ? j : 0);
          }
        }
        // (T % NSLOT == 0, so the ring slot of step s is t % NSLOT for every slice)
        if (t + 2 < T) issue_b(cb0 + cl, t + 2, (t + 2) % NSLOT);
        else if (cl + 1 < nsl) issue_b(cb0 + cl + 1, t + 2 - T, (t + 2) % NSLOT);
        MA_LAP(1, tl);
        // MFMA phase: A from the halo at the tap's pixel offset, B from ring slot s % 3
        const int r = t / R, ss = t % R;
        const int toff = g.HALF ? r * g.HWP + (ss >> 1) + (ss & 1) * g.HALF : r * g.HWP + ss;
        const int tsw = toff + g.SWA * r;                 // swizzle term of the tap's row
        const char* bs = ring + (t % NSLOT) * SLOT;
        // all 16 fragment reads of the tap first (both 32-deep halves in flight at once: one
        // wave per SIMD has no partner to hide LDS latency), then the MFMAs
        bf16x8 fa[2][TM], fb[2][TN];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const int chunk = kk * 4 + (lane >> 4);
#pragma unroll
          for (int tn = 0; tn < TN; ++tn) {
            const int row = wn * (BN / WN) + tn * 16 + (lane & 15);
            fb[kk][tn] = *(const bf16x8*)(bs + (row * 8 + (chunk ^ (row & 7))) * 16);
          }
#pragma unroll
          for (int tm = 0; tm < TM; ++tm) {
            const int p = apix[tm] + toff;
            fa[kk][tm] = *(const bf16x8*)(hb + (p * 8 + (chunk ^ ((aswz[tm] + tsw) & 7))) * 16);
          }
        }
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int tm = 0; tm < TM; ++tm)
#pragma unroll
            for (int tn = 0; tn < TN; ++tn)
              acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[kk][tn], fa[kk][tm],
                                                                   acc[tm][tn], 0, 0, 0);
        // keep that order: the scheduler otherwise re-serialises the reads (one fragment
        // register, an lgkmcnt(0) before every four MFMAs) to save registers it has plenty of
        __builtin_amdgcn_sched_group_barrier(0x100, 2 * (TM + TN), 0);   // DS reads
        __builtin_amdgcn_sched_group_barrier(0x008, 2 * TM * TN, 0);     // MFMAs
#ifdef MERCURY_STAMPS
        // (diagnostic build: make the MFMA phase's end observable)
        asm volatile("s_nop 0" ::"v"(acc[0][0]));
#endif
        MA_LAP(2, tl);
      }
    }
    vm_wait<0>();
  }
  MA_STAMP(2);
#ifdef MERCURY_STAMPS
  if (threadIdx.x == 0) {
    const int b_ = blockIdx.x + blockIdx.y * gridDim.x;
    if (b_ < 8192)
      for (int q = 0; q < 4; ++q) g_stamps[b_][4 + q] = lap[q];
  }
#endif
  __syncthreads();                                // LDS is reused by the epilogue
  finish<BM, BN, WM>(acc, smem, e, M, g.K, m0, n0, bx, by, gx, gy);
  MA_STAMP(3);
}

// ---------------------------------------------------------------- persistent variant
// One block per CU walks a strided list of output tiles as ONE continuous step stream
// (tile, 64-channel slice, tap), so the per-tile prologue (halo + first weight tiles from HBM)
// and the epilogue overlap the neighbouring tiles' MFMAs instead of serialising each block:
//   * the next slice's halo -- the next TILE's when this is a tile's last slice -- is issued in
//     pieces during taps 0..PHP-1 into the other of two halo buffers;
//   * weights run PDW = 5 steps ahead in a 6-slot ring (the single in-order vmcnt makes a
//     wait for a weight tile also wait for every older halo piece: 5 steps cover HBM latency);
//   * fragments of step s + 1 are read from LDS while step s's MFMAs execute;
//   * the epilogue stages through its own LDS area with raw barriers and issues a FIXED number
//     of stores / stat atomics per wave (E), so the following taps' counted waits stay exact
//     and nothing drains the in-flight DMAs.
// The tile-invariant part of each halo slot's source offset is computed once; a new tile only
// adds its (image, row) base.  Plain input only (MODE 0), no bias / accumulate / split-K, whole
// tiles (M % BM == 0, K % BN == 0, ghost-BN groups a multiple of BM): the host checks.
constexpr int PDW = 5;              // weight prefetch distance (steps)
constexpr int PSLOT = PDW + 1;      // weight ring slots
constexpr int PHP = 4;              // taps of a slice carrying the next slice's halo pieces

// Lean persistent epilogue (the default): the tile goes out as 8-byte buffer stores straight from
// the accumulators (lane l: output pixel l & 15, four consecutive channels) -- no LDS staging and
// no barrier -- and its ghost-BN sums are added to per-lane RUNNING sums.  The block walks a
// contiguous, N-tile-major range of tiles, so consecutive tiles share (statistics group, channel
// tile) and the cross-lane / cross-wave reduction and the global atomics (epi_flush) run once per
// (group, channel tile) the block touches instead of once per tile.  PMC, ResNet-18 scoring pass:
// the per-tile staged epilogue made the kernel 4.15 VALU per MFMA (profiles/r4/pmc).
// Weight-row order of the persistent kernels' ring with PERM: within every 32 rows, LDS row
// h * 16 + 4 q + j (fragment half h, lane group q, accumulator element j) holds channel
// 8 q + 4 h + j, so a lane's accumulators of fragments (2t, 2t + 1) are 8 consecutive channels
// of one pixel and leave as ONE 16-byte store (pgemm.hip pg_perm)
MA_DEV int hc_perm(int r) {
  const int r5 = r & 31;
  return (r & ~31) | (((r5 >> 2) & 3) << 3) | ((r5 >> 4) << 2) | (r5 & 3);
}

// stores per wave of one tile (the counted waits include them)
template <int BM, int BN, int WM, int NW, bool PERM>
constexpr int epi_stores() {
  return (BM / (16 * WM)) * (BN * WM / (16 * NW)) / (PERM ? 2 : 1);
}

template <int BM, int BN, int WM, int NW, bool PERM = false>
MA_DEV void epi_lean(const f32x4 (&acc)[BM / (16 * WM)][BN * WM / (16 * NW)],
                     float (&rs)[BN * WM / (16 * NW)][4], float (&rss)[BN * WM / (16 * NW)][4],
                     bool stats, const EpiParams& e, int m0, int n0, int vr) {
  constexpr int WN = NW / WM, TM = BM / (16 * WM), TN = BN / (16 * WN);
  static_assert(!PERM || TN % 2 == 0, "fragment pairs");
  typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w / WN, wn = w % WN;
  const auto ro = __builtin_amdgcn_make_buffer_rsrc((void*)e.out, 0, 0x7fffffff, 0x00020000);
  // tile row of this lane's fragment-0 pixel; rows >= vr pad a tile of whole image rows that
  // do not fill BM (56- / 28-wide images): their stores go past the resource (dropped) and
  // they add nothing to the statistics -- every wave still issues all its stores, so the
  // counted waits stay exact
  const int rl = wm * (BM / WM) + (lane & 15);
  if constexpr (PERM) {
    const unsigned voff =
        (unsigned)((((m0 + rl) * e.ldo) + n0 + wn * (BN / WN) + 8 * (lane >> 4)) * 2);
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
      const bool ok = rl + tm * 16 < vr;
#pragma unroll
      for (int tp = 0; tp < TN / 2; ++tp) {
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          o[j] = f2bf(acc[tm][2 * tp][j]);
          o[4 + j] = f2bf(acc[tm][2 * tp + 1][j]);
        }
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(u32x4, o), ro,
            ok ? voff + (unsigned)((tm * 16 * e.ldo + tp * 32) * 2) : 0x80000000u, 0, 0);
        if (stats) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float f = ok ? bf2f(o[j]) : 0.f, f2 = ok ? bf2f(o[4 + j]) : 0.f;
            rs[2 * tp][j] += f;
            rss[2 * tp][j] = fmaf(f, f, rss[2 * tp][j]);
            rs[2 * tp + 1][j] += f2;
            rss[2 * tp + 1][j] = fmaf(f2, f2, rss[2 * tp + 1][j]);
          }
        }
      }
    }
    return;
  }
  const unsigned voff = (unsigned)((((m0 + rl) * e.ldo) + n0 + wn * (BN / WN) + 4 * (lane >> 4)) * 2);
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const bool ok = rl + tm * 16 < vr;
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      bf16x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = f2bf(acc[tm][tn][j]);
      __builtin_amdgcn_raw_buffer_store_b64(
          __builtin_bit_cast(u32x2v, o), ro,
          ok ? voff + (unsigned)((tm * 16 * e.ldo + tn * 16) * 2) : 0x80000000u, 0, 0);
      if (stats) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float f = ok ? bf2f(o[j]) : 0.f;
          rs[tn][j] += f;
          rss[tn][j] = fmaf(f, f, rss[tn][j]);
        }
      }
    }
  }
}

// the running sums of (group g, channel tile n0) -> e.stats: DPP row sums, one LDS slot per
// (wave row, channel), one atomic pair per channel.  ``red``: 2 * WM * BN floats of LDS that no
// wave reads or DMAs into until the next slice's first barrier.  Block-uniform call.
template <int BM, int BN, int WM, int NW, bool PERM = false>
MA_DEV void epi_flush(float (&rs)[BN * WM / (16 * NW)][4], float (&rss)[BN * WM / (16 * NW)][4],
                      float* red, const EpiParams& e, int g, int n0) {
  constexpr int WN = NW / WM, TN = BN / (16 * WN);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w / WN, wn = w % WN;
#pragma unroll
  for (int tn = 0; tn < TN; ++tn)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      rs[tn][j] = row16_sum(rs[tn][j]);
      rss[tn][j] = row16_sum(rss[tn][j]);
    }
  bar_lds();                                        // every wave's reads of the area are done
  if ((lane & 15) == 0) {
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      float* r = red + wm * 2 * BN + wn * (BN / WN) +
                 (PERM ? (tn >> 1) * 32 + 8 * (lane >> 4) + 4 * (tn & 1) : tn * 16 + 4 * (lane >> 4));
      *(f32x4*)r = f32x4{rs[tn][0], rs[tn][1], rs[tn][2], rs[tn][3]};
      *(f32x4*)(r + BN) = f32x4{rss[tn][0], rss[tn][1], rss[tn][2], rss[tn][3]};
    }
  }
#pragma unroll
  for (int tn = 0; tn < TN; ++tn)
#pragma unroll
    for (int j = 0; j < 4; ++j) rs[tn][j] = rss[tn][j] = 0.f;
  bar_lds();
  if (tid < BN) {
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int q = 0; q < WM; ++q) {
      a += red[q * 2 * BN + tid];
      b += red[q * 2 * BN + BN + tid];
    }
    float* dst = MA_SPREAD(e.stats + (size_t)g * 2 * e.stats_ld + n0 + tid);
    atomicAdd(dst, a);
    atomicAdd(dst + e.stats_ld, b);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // red read before any later DMA lands
}

// raw buffer resource over [base, base + bytes): an LDS-DMA whose offset is past the end
// lands ZEROS (the padding halo pixels need no zero page and no second pointer)
MA_DEV __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, bytes, 0x00020000);
}
// 16 bytes per lane, buffer -> LDS (lane l lands at the wave-uniform LDS address + 16 l)
MA_DEV void bdma16(__amdgpu_buffer_rsrc_t r, unsigned off, unsigned lds) {
  // (readfirstlane: resource and base are wave-uniform; under register pressure the compiler
  // may otherwise hand the asm VGPRs for them)
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
               ::"v"(off), "s"(r), "s"(__builtin_amdgcn_readfirstlane(lds)) : "memory");
}
// the same DMA with the buffer resource assembled from (base, bytes) as four wave-uniform
// dwords (readfirstlane): where register pressure is high the compiler kept a resource built by
// __builtin_amdgcn_make_buffer_rsrc in VGPRs, which the asm cannot take
typedef unsigned u32x4s __attribute__((ext_vector_type(4)));
MA_DEV u32x4s rsrc_words(const void* base, unsigned bytes) {
  const unsigned long long a = (unsigned long long)base;
  u32x4s v;
  v[0] = __builtin_amdgcn_readfirstlane((unsigned)a);
  v[1] = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  v[2] = __builtin_amdgcn_readfirstlane(bytes);
  v[3] = 0x00020000u;
  return v;
}
MA_DEV void bdma16w(u32x4s r, unsigned off, unsigned lds) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
               ::"v"(off), "s"(r), "s"(__builtin_amdgcn_readfirstlane(lds)) : "memory");
}
constexpr unsigned OOB = 0x7ffffff0u;   // offset past every tensor: zeros

// vmcnt immediate at tap t: VMEM ops issued after step s + 1's weight tile (issued at step
// s + 1 - PDW) -- the issues of the PDW - 2 steps before s: BI weight pieces each (a step x of
// this slice issues for x + PDW, in the next slice when x + PDW >= T: only if one follows, hn),
// PHI halo pieces on carrying taps x < PHP of a slice that prefetches a halo (hd)
template <int t, int T, int BI, int PHI, bool hd, bool hn>
constexpr int tap_wait() {
  int n = 0;
  for (int x = t - (PDW - 2); x < t; ++x) {
    if (x < 0) {
      n += BI;
    } else {
      if (x + PDW < T || hn) n += BI;
      if (x < PHP && hd) n += PHI;
    }
  }
  return n;
}

// counted wait after which the epilogue's E VMEM ops (issued after the waited-for DMA) may be
// outstanding: E = ST stores + 2 stat atomics on the waves that issue them
template <int N, int ST, bool STATS>
MA_DEV void wait_epi(bool epi, bool ew) {
  if (!epi) vm_wait<N>();
  else if (STATS && ew) vm_wait<N + ST + 2>();
  else vm_wait<N + ST>();
}

// the wait of tap t (t is a constant once the tap loop is unrolled: the switch folds)
template <int T, int BI, int PHI, int ST, bool STATS>
MA_DEV void wait_tap(int t, bool hd, bool hn, bool epi, bool ew) {
  static_assert(T == 9, "3x3 taps");
#define WT(tt)                                                                              \
  case tt:                                                                                  \
    if (hd) {                                                                               \
      if (hn) wait_epi<tap_wait<tt, T, BI, PHI, true, true>(), ST, STATS>(epi, ew);         \
      else wait_epi<tap_wait<tt, T, BI, PHI, true, false>(), ST, STATS>(epi, ew);           \
    } else {                                                                                \
      if (hn) wait_epi<tap_wait<tt, T, BI, PHI, false, true>(), ST, STATS>(epi, ew);        \
      else wait_epi<tap_wait<tt, T, BI, PHI, false, false>(), ST, STATS>(epi, ew);          \
    }                                                                                       \
    break;
  switch (t) { WT(0) WT(1) WT(2) WT(3) WT(4) WT(5) WT(6) WT(7) WT(8) }
#undef WT
}

template <int BM, int BN, int WM, int NW, int NHB, int HRC, bool STATS, int MODE>
__global__ __launch_bounds__(64 * NW, 1) void hconv_persist_kernel(const bf16* __restrict__ src,
                                                              const bf16* __restrict__ wt,
                                                              HconvGeom g, EpiParams e,
                                                              HconvPro pro) {
  constexpr int NTP = 64 * NW;                      // threads (NW waves, one block per CU)
  constexpr int WN = NW / WM;
  constexpr int TM = BM / (16 * WM), TN = BN / (16 * WN);
  constexpr int PPX = 8 * NW;                       // halo pixels per DMA piece (8 per wave)
  constexpr int BI = BN / PPX;                      // weight DMA pieces per wave per step
  static_assert(BI >= 1 && BN % PPX == 0, "whole weight pieces per wave");
  constexpr int SLOT = BN * 128;
  constexpr int R = 3, T = R * R;
  // 16-byte epilogue stores from fragment pairs (hc_perm weight-row order) where TN is even
  constexpr bool PERM = TN % 2 == 0;
  constexpr int ST = epi_stores<BM, BN, WM, NW, PERM>();   // epilogue stores per wave
  constexpr int PHI = HRC / PHP;                    // halo pieces per wave on a carrying tap
  static_assert(PHP <= T - 3, "a slice's halo lands >= 2 steps before its first read");
  static_assert(HRC % PHP == 0 && HRC <= HRMAX, "halo piece capacity");
  static_assert(MODE == 0 || MODE == 1, "persistent kernel: plain or BN + activation input");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w / WN, wn = w % WN;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const bool ew = wu * 64 < BN;                     // this wave issues the stat atomics
  const int ntn = g.K / BN;
  const int PQ = g.P * g.Q;
  // output rows per tile: IMG whole images or TR whole rows of one image -- BM, or fewer when
  // no whole-row count fills BM (56- / 28-wide images: 2 x 56 or 4 x 28 = 112 of 128 rows; the
  // remaining fragment rows are computed on a clamped halo pixel and dropped in epi_lean)
  const int VR = g.IMG * g.TR * g.Q;
  const int ntiles = (g.N * PQ / VR) * ntn;
  const int G = gridDim.x, b = blockIdx.x;
  // a contiguous range of tiles per block, N-tile-major (consecutive tiles share their channel
  // tile and, mostly, their statistics group: epi_lean's running sums)
  const int mtiles = g.N * PQ / VR;
  const int t0 = (int)((long long)ntiles * b / G);
  const int my = (int)((long long)ntiles * (b + 1) / G) - t0;
  if (my == 0) return;
  MA_STAMP(0);
#ifdef MERCURY_STAMPS
  // per-step phase sums of wave 0 (shader clocks): [0] first MFMA half issue, [1] vmcnt wait,
  // [2] barrier, [3] DMA issue, [4] reads + second MFMA half, [5] epilogue
  unsigned long long lap[6] = {0, 0, 0, 0, 0, 0};
  unsigned long long tl = __builtin_amdgcn_s_memtime();
#endif
  const int nsl = g.C >> 6;
  const int Kt = T * g.C;
  const int HR = (g.HPIX + PPX - 1) / PPX;
  const int HBYTES = HR * PPX * 128;
  const int lc = (lane & 7) ^ (lane >> 3);
  const int per_img = g.HT * g.HWP;
  const auto rs_src = buf_rsrc(src, (unsigned)((size_t)g.N * g.H * g.W * g.C * 2));
  const auto rs_wt = buf_rsrc(wt, (unsigned)((size_t)g.K * Kt * 2));

  // ---- tile-invariant halo slots: byte offset from the tile's (image, row) base, and the
  // slot's input-row step (HROW_NONE for padding columns / unused slots: never in range).
  // The host keeps N a multiple of IMG, so only the row test depends on the tile.
  constexpr int HROW_NONE = 0x4000;
  int hbase[HRC], hrow[HRC];
#pragma unroll
  for (int i = 0; i < HRC; ++i) {
    hbase[i] = 0;
    hrow[i] = HROW_NONE;
    const int pix = (tid >> 3) + PPX * i;
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
      const int ww = hc * g.HS - g.pad;
      if (ok && (unsigned)ww < (unsigned)g.W) {
        hbase[i] = (((img * g.H + hr * g.HS) * g.W + ww) * g.C + lc * 8) * 2;
        hrow[i] = hr * g.HS;
      }
    }
  }
  unsigned hoff[HRC];                                // byte offsets of the current halo (OOB: pad)
  int hgrp = 0;                                      // ... and its statistics group (MODE 1)
  const float rmt = 1.f / (float)mtiles, rpq = 1.f / (float)PQ, rq = 1.f / (float)g.Q;
  auto tile_of = [&](int k, int& m0, int& n0) {
    const int t = t0 + k;
    const int nt = udiv24(t, mtiles, rmt), mt = t - nt * mtiles;
    m0 = mt * VR;
    n0 = nt * BN;
  };
  auto set_halo = [&](int m0) {
    const int n0i = udiv24(m0, PQ, rpq);
    const int p0 = udiv24(m0 - n0i * PQ, g.Q, rq);
    const int h0 = p0 * g.stride - g.pad;
    const int toff = (n0i * g.H + h0) * g.W * g.C * 2;
    if constexpr (MODE == 1) hgrp = n0i / pro.group_imgs;   // a tile's images share a group
#pragma unroll
    for (int i = 0; i < HRC; ++i)
      hoff[i] = (unsigned)(h0 + hrow[i]) < (unsigned)g.H ? (unsigned)(hbase[i] + toff) : OOB;
  };
  // A-fragment byte offsets in a halo buffer, per (tap, fragment row block): the swizzled chunk
  // of the k = 0..31 half (the other half is the same ^ 64)
  const int c16 = (lane >> 4) << 4;
  int aoff[T][TM];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int rowt = wm * (BM / WM) + tm * 16 + (lane & 15);
    const int row = rowt < VR ? rowt : 0;           // padding rows: a real pixel, result dropped
    const int img = row / (g.TR * g.Q), rem = row - img * g.TR * g.Q;
    const int tr = rem / g.Q, q = rem - tr * g.Q;
    const int hc = q * g.SR;
    const int col = g.HALF ? ((hc & 1) * g.HALF + (hc >> 1)) : hc;
    const int apix = img * per_img + tr * g.SR * g.HWP + col;
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int r = t / R, ss = t % R;
      const int p = apix + (g.HALF ? r * g.HWP + (ss >> 1) + (ss & 1) * g.HALF : r * g.HWP + ss);
      aoff[t][tm] = (p << 7) + (c16 ^ ((p & 7) << 4));
    }
  }
  unsigned boff[BI];                                 // weight rows this lane fetches (bytes)
#pragma unroll
  for (int j = 0; j < BI; ++j) {
    const int r = 8 * (w + NW * j) + (lane >> 3);  // ring row; the channel it holds:
    boff[j] = (((PERM ? hc_perm(r) : r)) * Kt + lc * 8) * 2;
  }
  // B-fragment byte offsets inside a ring slot (tap-invariant)
  int bfo[2][TN];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int row = wn * (BN / WN) + tn * 16 + (lane & 15);
      bfo[kk][tn] = (row * 8 + ((kk * 4 + (lane >> 4)) ^ (row & 7))) * 16;
    }
  const unsigned s_halo = lds_addr(smem);
  const unsigned s_ring = s_halo + NHB * HBYTES;
  const unsigned s_dump = s_ring + PSLOT * SLOT + wu * 1024;      // 1 KB per wave
  // MODE 1: per-(statistics group, 8-channel chunk) BN scale[8] | shift[8] of the input, built
  // once per block in LDS, so the halo transform reads no global memory (a compiler-visible
  // load there would make hipcc drain every in-flight DMA)
  float* const coef = (float*)(smem + NHB * HBYTES + PSLOT * SLOT + NW * 1024);
  float csc[8], csh[8];                               // this thread's chunk of the slice

  // in-place BN + activation of this thread's own DMA'd chunks (pieces j0 <= j < j1) of a landed
  // halo (buffer hb_i, 64-channel slice cb, statistics group grp); padding pixels stay zero
  auto xform = [&](int hb_i, int j0, int j1) {
    if constexpr (MODE == 1) {
      float lo, hi;
      act_bounds(pro.act, lo, hi);
      char* hb = smem + hb_i * HBYTES + (tid >> 3) * 128 + (tid & 7) * 16;
#pragma unroll
      for (int j = 0; j < HRC; ++j) {
        if (j < j0 || j >= j1 || j >= HR || hoff[j] == OOB) continue;
        u32x4* lp = (u32x4*)(hb + j * PPX * 128);
        const bf16x8 y = __builtin_bit_cast(bf16x8, *lp);
        bf16x8 o;
#pragma unroll
        for (int q = 0; q < 8; ++q) o[q] = f2bf(fminf(fmaxf(bf2f(y[q]) * csc[q] + csh[q], lo), hi));
        *lp = __builtin_bit_cast(u32x4, o);
      }
    }
  };
  auto load_coef_lds = [&](int cb, int grp) {
    if constexpr (MODE == 1) {
      const f32x4* c = (const f32x4*)(coef + ((size_t)grp * (g.C >> 3) + cb * 8 + lc) * 16);
      const f32x4 a = c[0], b2 = c[1], d = c[2], f = c[3];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        csc[q] = a[q];
        csc[4 + q] = b2[q];
        csh[q] = d[q];
        csh[4 + q] = f[q];
      }
    }
  };

  auto issue_h = [&](int cb, int buf, int j) {
    // (HR through an empty asm: hoisted, the 16 `j < HR` tests were kept as lane masks and
    // spilled to VGPR lanes)
    int hr = HR;
    asm volatile("" : "+s"(hr));
    bdma16(rs_src, hoff[j] + cb * 128, j < hr ? s_halo + buf * HBYTES + (PPX * j + 8 * wu) * 128
                                              : s_dump);
  };
  auto issue_b = [&](int n0, int cb, int t, int slot) {
    const unsigned k = (unsigned)((n0 * Kt + t * g.C + cb * 64) * 2);
#pragma unroll
    for (int j = 0; j < BI; ++j)
      bdma16(rs_wt, boff[j] + k, s_ring + slot * SLOT + 8 * (wu + NW * j) * 128);
  };
  // fragments of (halo buffer, ring slot, tap); the k = 0..31 half first (the next step's
  // first MFMAs need only that)
  auto read_frags = [&](bf16x8 (&fa)[2][TM], bf16x8 (&fb)[2][TN], int hbuf, int slot, int tap) {
    const char* bs = smem + NHB * HBYTES + slot * SLOT;
    const char* hb = smem + hbuf * HBYTES;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) fa[0][tm] = *(const bf16x8*)(hb + aoff[tap][tm]);
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) fb[0][tn] = *(const bf16x8*)(bs + bfo[0][tn]);
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
      fa[1][tm] = *(const bf16x8*)(hb + (aoff[tap][tm] ^ 64));   // chunk + 4 = swizzled ^ 4
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) fb[1][tn] = *(const bf16x8*)(bs + bfo[1][tn]);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float rsum[TN][4], rsq[TN][4];                     // running ghost-BN sums (epi_lean)
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) rsum[i][j] = rsq[i][j] = 0.f;

  // ---- slice cursors.  Slice sigma = (tile k, 64-channel slice cl); the block walks
  // NS = my * nsl of them.  Halo of slice sigma + D (D = NHB - 1) is prefetched during slice
  // sigma into buffer (sigma + D) % NHB, the weights of the next slice during its last taps.
  constexpr int D = NHB - 1;
  const int NS = my * nsl;
  int m0, n0;                                        // tile of the current slice
  tile_of(0, m0, n0);
  int kD = 0, clD = 0;                               // slice whose halo hoff describes
  auto advance_d = [&]() {                           // kD, clD -> next slice (+ its halo slots)
    if (++clD == nsl) {
      clD = 0;
      if (++kD < my) {
        int mD, nD;
        tile_of(kD, mD, nD);
        set_halo(mD);
      }
    }
  };
  // ---- prologue: the BN table (MODE 1), slice 0's halo, weight tiles of steps 0..PDW-1,
  // fragments of step 0
  static_assert(D == 1, "one halo prefetched ahead");
  static_assert(PDW < T, "prologue weight tiles lie in slice 0");
  if constexpr (MODE == 1) {
    const int G = pro.stats ? g.N / pro.group_imgs : 1;
    for (int i = tid; i < G * g.C; i += NTP) {
      const int gi = i / g.C, c = i - gi * g.C;
      float mean, var;
      if (pro.stats) {
        mean = pro.stats[(size_t)gi * 2 * g.C + c] * pro.inv_count;
        var = fmaxf(pro.stats[(size_t)gi * 2 * g.C + g.C + c] * pro.inv_count - mean * mean, 0.f);
      } else {
        mean = pro.rmean[c];
        var = pro.rvar[c];
      }
      const float sc = pro.gamma[c] * rsqrtf(var + pro.eps);
      float* t = coef + ((size_t)gi * (g.C >> 3) + (c >> 3)) * 16 + (c & 7);
      t[0] = sc;
      t[8] = pro.beta[c] - mean * sc;
    }
  }
  set_halo(m0);
#pragma unroll
  for (int j = 0; j < HRC; ++j)
    if (j < HR) issue_h(0, 0, j);
#pragma unroll
  for (int t = 0; t < PDW; ++t) issue_b(n0, 0, t, t);
  vm_wait<0>();
  if constexpr (MODE == 1) {
    bar_lds();                                        // the table is complete
    load_coef_lds(0, hgrp);
    xform(0, 0, HRC);
  }
  advance_d();                                        // (kD, clD) = slice 1: prefetched in slice 0
  bar_lds();
  bf16x8 fa[2][TM], fb[2][TN];
  read_frags(fa, fb, 0, 0, 0);
  MA_STAMP(1);

  constexpr int NM = TM * TN;
  // MFMAs [i0, i1) of half kk of the current step (fragments already in registers)
  auto mma = [&](int kk, int i0, int i1) {
#pragma unroll
    for (int i = 0; i < NM; ++i)
      if (i >= i0 && i < i1)
        acc[i / TN][i % TN] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            fb[kk][i % TN], fa[kk][i / TN], acc[i / TN][i % TN], 0, 0, 0);
  };

  // Step s (tap t of a slice): wait for step s + 1's weight tile, barrier, read step s + 1's
  // fragments, issue the DMAs of step s + PDW and this slice's share of halo pieces.  The 2 NM
  // MFMAs of step s are spread over all of it (the wait, the barrier and every DMA issue stall
  // the wave; MFMAs issued before them keep the matrix pipe busy).  Newer than the awaited tile
  // at the wait: tap_wait() pieces and, on taps <= PDW - 2 of a tile's first slice, the
  // previous tile's epilogue (E) -- every count is a compile-time immediate per tap.
  int s0 = 0, cl = 0, k = 0, buf = 0, bufD = D % NHB, sb = 0;   // sb = s0 % PSLOT
  for (int sig = 0; sig < NS; ++sig, s0 += T) {
    const bool last_sl = cl + 1 == nsl;
    const bool hn = sig + 1 < NS;                    // a slice follows this one
    const bool hd = sig + D < NS;                    // this slice prefetches a halo
    int m0n = m0, n0n = n0;
    const int cbn = last_sl ? 0 : cl + 1;
    if (last_sl && hn) tile_of(k + 1, m0n, n0n);
    const bool epi = cl == 0 && k > 0;
    const int cbD = clD;
    const int bnext = buf + 1 == NHB ? 0 : buf + 1;
    auto slot_of = [&](int u) {                      // ring slot of step s0 + u, u < 2 PSLOT
      const int v = sb + u;
      return v >= 2 * PSLOT ? v - 2 * PSLOT : (v >= PSLOT ? v - PSLOT : v);
    };
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const bool go = t < T - 1 || hn;               // step s + 1 exists
      mma(0, 0, NM / 2);
      MA_LAP(0, tl);
      if (go) {
        wait_tap<T, BI, PHI, ST, STATS>(t, hd, hn, epi && t <= PDW - 2, false);
      }
      MA_LAP(1, tl);
      if constexpr (MODE == 1) {
        // the next slice's halo pieces issued at tap t - (PDW - 1) have landed (this wave's
        // own): normalise them in place; the tap-(T-1) barrier publishes the writes
        constexpr int XT = PDW - 1;
        static_assert(XT + PHP <= T - 1, "transform before the last tap's barrier");
        if (hd && t >= XT && t < XT + PHP) {
          if (t == XT) load_coef_lds(cbD, hgrp);
          xform(bufD, (t - XT) * PHI, (t - XT + 1) * PHI);
        }
      }
      mma(0, NM / 2, 3 * NM / 4);
      if (go) {
        if (MODE == 1 && t == T - 1) bar_lds();
        else bar_raw();
      }
      MA_LAP(2, tl);
      mma(0, 3 * NM / 4, NM);
      if (go) {
        if (hd && t < PHP) {
#pragma unroll
          for (int q = 0; q < PHI; ++q) issue_h(cbD, bufD, t * PHI + q);
        }
        if (t + PDW < T) issue_b(n0, cl, t + PDW, slot_of(t + PDW));
        else if (hn) issue_b(n0n, cbn, t + PDW - T, slot_of(t + PDW));
      }
      MA_LAP(3, tl);
      bf16x8 na[2][TM], nb[2][TN];
      // step s + 1's fragments interleaved with the k = 32..63 half of step s (unconditional,
      // so reads and MFMAs share one basic block; the block's last step reads a stale slot it
      // never uses).  (Reading them right after the barrier instead measured slower: 1.545 vs
      // 1.526 ms/step, layer1 40.2 vs 38.7 us.)
      read_frags(na, nb, t + 1 < T ? buf : bnext, slot_of(t + 1), t + 1 < T ? t + 1 : 0);
      mma(1, 0, NM);
      constexpr int NR = 2 * (TM + TN);
      constexpr int RPM = (NR + NM - 1) / NM;        // reads per MFMA gap
#pragma unroll
      for (int i = 0; i < NM; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x100, RPM, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) fa[kk][tm] = na[kk][tm];
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) fb[kk][tn] = nb[kk][tn];
      }
#ifdef MERCURY_STAMPS
      asm volatile("s_nop 0" ::"v"(acc[0][0]));
#endif
      MA_LAP(4, tl);
      if (t == T - 1 && last_sl) {
        // staged in this slice's halo buffer: fully read, refilled only from the next slice on
        epi_lean<BM, BN, WM, NW, PERM>(acc, rsum, rsq, STATS, e, m0, n0, VR);
        if (STATS) {
          // flush when the next tile of this block starts another (group, channel tile)
          const int gcur = m0 / e.group_rows;
          if (!hn || n0n != n0 || m0n / e.group_rows != gcur)
            epi_flush<BM, BN, WM, NW, PERM>(rsum, rsq, (float*)(smem + buf * HBYTES), e, gcur,
                                            n0);
        }
        MA_LAP(5, tl);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    // next slice; the halo cursor moves to the slice after the one just prefetched (its slots
    // are recomputed only here, after this slice's last halo piece was issued)
    if (hd) advance_d();
    m0 = m0n;
    n0 = n0n;
    buf = bnext;
    bufD = bufD + 1 == NHB ? 0 : bufD + 1;
    sb = (sb + T) % PSLOT;
    if (last_sl) {
      cl = 0;
      ++k;
    } else {
      ++cl;
    }
  }
  MA_STAMP(2);
#ifdef MERCURY_STAMPS
  if (threadIdx.x == 0 && blockIdx.x < 8192)
    for (int q = 0; q < 6; ++q) g_stamps[blockIdx.x][4 + q] = lap[q];
#endif
  MA_STAMP(3);
}

// ---------------------------------------------------------------- row-step persistent variant
// The scoring pass's stride-1 3x3 convs (B = 320, SURVEY K5 / `pytorch_collab.py:95-103`).
// hconv_persist synchronises its waves once per TAP (a 64-deep K step): its phase stamps put the
// per-tap barrier at 433 cycles against 440 of MFMA issue (profiles/r4/stamps).  Here one STEP
// is one filter ROW -- 3 taps x 64 channels, K = 192 -- so a block synchronises three times per
// 64-channel slice, and each wave issues 6 sub-steps of TM x TN MFMAs per barrier:
//   * weights: a ring of WS slots, each one filter row (3 taps x BN channel rows x 64 channels,
//     the igemm image [row][64] with chunk c ^ (row & 7)); the row of step s + 1 is DMA'd during
//     step s (weights are L2-resident: one step of ~1.5k cycles covers them);
//   * STATIONARY (C = K = 64, ResNet layer1: one slice, one channel tile): the three filter
//     rows fill the three slots once and stay for the block's life, so the only staged operand
//     is the halo and a block synchronises once per TILE;
//   * halo: the next slice's (the next tile's when the slice is a tile's last) is DMA'd in two
//     halves during rows 0 and 1 of the current slice, AFTER that step's weight row: the wait
//     for a weight row therefore never waits for an HBM halo piece issued in the same step,
//     and a halo is waited for only at its own slice start (2-3 steps after issue);
//   * waits are counted (`s_waitcnt vmcnt(N)`, N a per-row immediate); the epilogue's stores
//     are the youngest VMEM ops at a slice start, so they never drain;
//   * pieces past the halo's last re-issue the last real piece (same source, same LDS bytes),
//     so every wave issues exactly HRC pieces per halo without a dump area (layer1's LDS is
//     exactly 160 KiB: two 44 KiB halos + three 24 KiB weight rows).
// Output layout, ghost-BN running sums and flushes are hconv_persist's (epi_lean / epi_flush).
template <int BM, int BN, int WM, int NW, int HRC, bool STATS, bool STAT, int MODE>
__global__ __launch_bounds__(64 * NW, 1) void hrow_kernel(const bf16* __restrict__ src,
                                                         const bf16* __restrict__ wt, HconvGeom g,
                                                         EpiParams e, HconvPro pro) {
  constexpr int WN = NW / WM;
  constexpr int TM = BM / (16 * WM), TN = BN / (16 * WN);
  constexpr int WROWS = 3 * BN;                     // weight rows per step (3 taps x BN)
  static_assert(WROWS % (8 * NW) == 0, "whole weight pieces per wave");
  constexpr int BI = WROWS / (8 * NW);              // weight DMA pieces per wave per step
  constexpr int WSLOT = WROWS * 128;                // bytes per ring slot
  static_assert(HRC % 2 == 0 && HRC <= HRMAX, "halo pieces split over rows 0 and 1");
  constexpr int HH = HRC / 2;                       // halo pieces per wave on rows 0 and 1
  constexpr bool PERM = TN % 2 == 0;                // 16-byte epilogue stores (hc_perm rows)
  constexpr int ST = epi_stores<BM, BN, WM, NW, PERM>();   // epilogue stores per wave
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w / WN, wn = w % WN;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const int ntn = g.K / BN;
  const int PQ = g.P * g.Q;
  const int mtiles = g.N * PQ / BM;
  const int ntiles = mtiles * ntn;
  const int G = gridDim.x, b = blockIdx.x;
  // a contiguous, N-tile-major range of tiles per block (epi_lean's running sums; STATIONARY:
  // one channel tile for the whole range)
  const int t0 = (int)((long long)ntiles * b / G);
  const int my = (int)((long long)ntiles * (b + 1) / G) - t0;
  if (my == 0) return;
  const int nsl = g.C >> 6;
  const int Kt = 9 * g.C;
  // halo: 8-pixel pieces; piece q of the halo is wave q % NW's (q / NW)-th.  A wave's issues
  // past its last real piece repeat that piece (same source, same LDS bytes), so every wave
  // issues exactly HRC per halo and the buffer holds just the halo (host: pieces <= HRC)
  const int HP8 = (g.HPIX + 7) >> 3;
  const int HBYTES = HP8 * 8 * 128;
  const int ilast = __builtin_amdgcn_readfirstlane((HP8 - 1 - wu) / NW);
  const int lc = (lane & 7) ^ (lane >> 3);
  const int per_img = g.HT * g.HWP;
  const unsigned src_bytes = (unsigned)((size_t)g.N * g.H * g.W * g.C * 2);
  const unsigned wt_bytes = (unsigned)((size_t)g.K * Kt * 2);

  // ---- tile-invariant halo slots, one register each: byte offset from the tile's (image, row)
  // base in the low 26 bits, the slot's input row above (63: padding column / beyond the halo;
  // host: a tile's images are < 64 MiB of input and < 63 halo rows)
  unsigned hslot[HRC];
#pragma unroll
  for (int i = 0; i < HRC; ++i) {
    hslot[i] = 63u << 26;
    const int pix = 8 * (w + NW * min(i, ilast)) + (lane >> 3);
    if (pix < g.HPIX) {
      const int img = pix / per_img, rem = pix - img * per_img;
      const int hr = rem / g.HWP, col = rem - hr * g.HWP;
      const int ww = col - g.pad;
      if (col < g.HWd && (unsigned)ww < (unsigned)g.W)
        hslot[i] = ((unsigned)hr << 26) | (unsigned)((((img * g.H + hr) * g.W + ww) * g.C + lc * 8) * 2);
    }
  }
  unsigned hoff[HRC];
  int hgrp = 0;                                      // statistics group of that halo (MODE 1)
  const float rmt = 1.f / (float)mtiles, rpq = 1.f / (float)PQ, rq = 1.f / (float)g.Q;
  auto tile_of = [&](int k, int& m0, int& n0) __attribute__((always_inline)) {
    const int t = t0 + k;
    const int nt = udiv24(t, mtiles, rmt), mt = t - nt * mtiles;
    m0 = mt * BM;
    n0 = nt * BN;
  };
  auto set_halo = [&](int m0) __attribute__((always_inline)) {
    const int n0i = udiv24(m0, PQ, rpq);
    const int p0 = udiv24(m0 - n0i * PQ, g.Q, rq);
    const int h0 = p0 - g.pad;
    const int toff = (n0i * g.H + h0) * g.W * g.C * 2;
    if constexpr (MODE >= 1) hgrp = pro.stats ? n0i / pro.group_imgs : 0;
#pragma unroll
    for (int i = 0; i < HRC; ++i) {
      const int hr = (int)(hslot[i] >> 26);
      hoff[i] = hr != 63 && (unsigned)(h0 + hr) < (unsigned)g.H
                    ? (hslot[i] & 0x3ffffffu) + (unsigned)toff : OOB;
    }
  };
  // MODE 1 / 2: the input is the producer's raw conv output; its BatchNorm (ghost-group batch or
  // running statistics) + activation is applied in LDS to each landed halo piece, once, by the
  // thread whose DMA brought it (8 channels lc of the slice: scale / shift loaded into registers
  // right before the transform, in the last row of the slice before).  Padding stays zero.
  // MODE 1 loads the statistics from global memory per slice; MODE 2 (the launcher's choice when
  // it fits: pro.coef_tab) reads scale / shift of the block's at most two statistics groups, ga
  // and gb, from a table built once in the prologue into LDS after the weight ring --
  // [2][C/8][scale 8 | shift 8] -- so the per-slice load is 4 LDS reads, not an exposed global
  // round trip (layer 1 64.8 -> 62.1-62.6 us, layer 2 66.7-67.1 -> 60.2-60.4, profiles/r5/hrow_mode1)
  float csc[8], csh[8];
  float* const ctab = (float*)(smem + 2 * HBYTES + (STAT ? 3 : 2) * WSLOT);
  int ga = 0, gb = 0;
  auto load_coef = [&](int cb, int grp) __attribute__((always_inline)) {
    if constexpr (MODE == 2) {
      const int slot = __builtin_amdgcn_readfirstlane(grp == ga ? 0 : (g.C >> 3));
      const f32x4* c = (const f32x4*)(ctab + (slot + cb * 8 + lc) * 16);
      const f32x4 a = c[0], b2 = c[1], d = c[2], f = c[3];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        csc[q] = a[q];
        csc[4 + q] = b2[q];
        csh[q] = d[q];
        csh[4 + q] = f[q];
      }
      return;
    }
    if constexpr (MODE == 1) {
      const int ch = cb * 64 + lc * 8;
      f32x4 a0, a1, b0, b1;
      if (pro.stats) {
        const float* st = pro.stats + (size_t)grp * 2 * g.C + ch;
        a0 = *(const f32x4*)st;
        a1 = *(const f32x4*)(st + 4);
        b0 = *(const f32x4*)(st + g.C);
        b1 = *(const f32x4*)(st + g.C + 4);
      } else {
        a0 = *(const f32x4*)(pro.rmean + ch);
        a1 = *(const f32x4*)(pro.rmean + ch + 4);
        b0 = *(const f32x4*)(pro.rvar + ch);
        b1 = *(const f32x4*)(pro.rvar + ch + 4);
      }
      const f32x4 g0 = *(const f32x4*)(pro.gamma + ch), g1 = *(const f32x4*)(pro.gamma + ch + 4);
      const f32x4 e0 = *(const f32x4*)(pro.beta + ch), e1 = *(const f32x4*)(pro.beta + ch + 4);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float a = q < 4 ? a0[q] : a1[q - 4], bb = q < 4 ? b0[q] : b1[q - 4];
        float mean = a, var = bb;
        if (pro.stats) {
          mean = a * pro.inv_count;
          var = fmaxf(bb * pro.inv_count - mean * mean, 0.f);
        }
        csc[q] = (q < 4 ? g0[q] : g1[q - 4]) * rsqrtf(var + pro.eps);
        csh[q] = (q < 4 ? e0[q] : e1[q - 4]) - mean * csc[q];
      }
    }
  };
  auto xform = [&](int hbuf) __attribute__((always_inline)) {
    if constexpr (MODE >= 1) {
      float lo, hi;
      act_bounds(pro.act, lo, hi);
#pragma unroll
      for (int i = 0; i < HRC; ++i) {
        if (i > ilast || hoff[i] == OOB) continue;   // (a repeat of piece ilast; padding)
        u32x4* lp = (u32x4*)(smem + hbuf * HBYTES + 8 * (w + NW * i) * 128 + lane * 16);
        const bf16x8 y = __builtin_bit_cast(bf16x8, *lp);
        bf16x8 o;
#pragma unroll
        for (int q = 0; q < 8; ++q) o[q] = f2bf(fminf(fmaxf(bf2f(y[q]) * csc[q] + csh[q], lo), hi));
        *lp = __builtin_bit_cast(u32x4, o);
      }
    }
  };
  // A-fragment byte offsets in a halo buffer per (tap, fragment row block), k = 0..31 half (the
  // other half is ^ 64)
  const int c16 = (lane >> 4) << 4;
  int aoff[9][TM];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int row = wm * (BM / WM) + tm * 16 + (lane & 15);
    const int img = row / (g.TR * g.Q), rem = row - img * g.TR * g.Q;
    const int tr = rem / g.Q, q = rem - tr * g.Q;
    const int apix = img * per_img + tr * g.HWP + q;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int p = apix + (t / 3) * g.HWP + t % 3;
      aoff[t][tm] = (p << 7) + (c16 ^ ((p & 7) << 4));
    }
  }
  // weight DMA: piece q of this wave = step rows 8 (w + NW q) .. + 8; lane -> row + lane >> 3
  unsigned boff[BI];
#pragma unroll
  for (int q = 0; q < BI; ++q) {
    const int row = 8 * (w + NW * q) + (lane >> 3);
    const int j = row / BN, n = row - j * BN;      // (tap, ring row); the channel it holds:
    boff[q] = (unsigned)(((PERM ? hc_perm(n) : n) * Kt + j * g.C + lc * 8) * 2);
  }
  // B-fragment byte offsets inside a slot, tap 0 of the row (tap j adds j * BN * 128)
  int bfo[2][TN];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int n = wn * (BN / WN) + tn * 16 + (lane & 15);
      bfo[kk][tn] = n * 128 + (((kk * 4 + (lane >> 4)) ^ (n & 7)) << 4);
    }
  const unsigned s_halo = lds_addr(smem);
  const unsigned s_ring = s_halo + 2 * HBYTES;

  auto issue_h = [&](int cb, int buf, int i) __attribute__((always_inline)) {
    const unsigned dst = __builtin_amdgcn_readfirstlane(
        s_halo + buf * HBYTES + 8 * (wu + NW * min(i, ilast)) * 128);
    bdma16w(rsrc_words(src, src_bytes), hoff[i] + cb * 128, dst);
  };
  // filter row r of (channel tile n0, slice cb) into ring slot `slot`
  auto issue_w = [&](int n0, int cb, int r, int slot) __attribute__((always_inline)) {
    const unsigned k = (unsigned)((n0 * Kt + 3 * r * g.C + cb * 64) * 2);
    const unsigned base = __builtin_amdgcn_readfirstlane(s_ring + slot * WSLOT + 8 * wu * 128);
#pragma unroll
    for (int q = 0; q < BI; ++q)
      bdma16w(rsrc_words(wt, wt_bytes), boff[q] + k, base + 8 * NW * q * 128);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float rsum[TN][4], rsq[TN][4];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) rsum[i][j] = rsq[i][j] = 0.f;

  // ---- slice cursors: slice sig = (tile k, slice cl); the halo cursor (kD, clD) is one ahead
  const int NS = my * nsl;
  int m0, n0;
  tile_of(0, m0, n0);
  int kD = 0, clD = 0;
  auto advance_d = [&]() __attribute__((always_inline)) {
    if (++clD == nsl) {
      clD = 0;
      if (++kD < my) {
        int mD, nD;
        tile_of(kD, mD, nD);
        set_halo(mD);
      }
    }
  };
  // ---- prologue: slice 0's halo and the first weight row(s), all landed
  set_halo(m0);
#pragma unroll
  for (int j = 0; j < HRC; ++j) issue_h(0, 0, j);
  if constexpr (STAT) {
#pragma unroll
    for (int r = 0; r < 3; ++r) issue_w(n0, 0, r, r);
  } else {
    issue_w(n0, 0, 0, 0);
  }
  if constexpr (MODE == 2) {
    int mA, nA, mB, nB;
    tile_of(0, mA, nA);
    tile_of(my - 1, mB, nB);
    if (pro.stats) {
      ga = __builtin_amdgcn_readfirstlane(udiv24(mA, PQ, rpq) / pro.group_imgs);
      gb = __builtin_amdgcn_readfirstlane(udiv24(mB, PQ, rpq) / pro.group_imgs);
    }
    for (int i = tid; i < 2 * g.C; i += 64 * NW) {
      const int sl = i >= g.C, c = i - sl * g.C, gi = sl ? gb : ga;
      float mean, var;
      if (pro.stats) {
        mean = pro.stats[(size_t)gi * 2 * g.C + c] * pro.inv_count;
        var = fmaxf(pro.stats[(size_t)gi * 2 * g.C + g.C + c] * pro.inv_count - mean * mean, 0.f);
      } else {
        mean = pro.rmean[c];
        var = pro.rvar[c];
      }
      const float sc = pro.gamma[c] * rsqrtf(var + pro.eps);
      float* t = ctab + (sl * (g.C >> 3) + (c >> 3)) * 16 + (c & 7);
      t[0] = sc;
      t[8] = pro.beta[c] - mean * sc;
    }
  }
  vm_wait<0>();
  if constexpr (MODE >= 1) {
    if (MODE == 2) bar_lds();                     // the table is complete
    load_coef(0, hgrp);
    xform(0);
  }
  advance_d();                                       // the halo cursor is at slice 1
  bar_lds();

  int cl = 0, k = 0, sb = 0;                         // sb: ring slot of this slice's row 0
  for (int sig = 0; sig < NS; ++sig) {
    const bool last_sl = cl + 1 == nsl;
    const bool hd = sig + 1 < NS;                    // a next slice exists: prefetch its halo
    const bool epi_prev = cl == 0 && k > 0;          // the previous slice ended a tile
    int m0n = m0, n0n = n0;
    const int cbn = last_sl ? 0 : cl + 1;
    if (last_sl && hd) tile_of(k + 1, m0n, n0n);
    const int buf = sig & 1;
    const int cbD = clD;
    const char* hb = smem + buf * HBYTES;

    // row r's start: its weight row (and, at r = 0, this slice's halo) has landed everywhere;
    // then the next row's weights and this row's share of the next slice's halo are issued.
    // Row 0 syncs before any read of this slice; rows 1 and 2 sync before the LAST tap of the
    // previous row computes (its fragments are in registers: bar_lds retires their reads
    // before the ring slot they came from is refilled)
    auto row_start = [&](int r) __attribute__((always_inline)) {
      if constexpr (STAT) {
        if (r == 0 && sig > 0) {
          vm_wait<ST>();                             // only the last tile's stores may be newer
          bar_lds();
        }
        if (MODE >= 1 && r == 2 && hd) {
          vm_wait<0>();                              // the next slice's halo has landed
          load_coef(cbD, hgrp);
          xform(buf ^ 1);
        }
        // (plain input too: draining the next halo here, two rows after its first pieces were
        // issued, instead of at the next slice's row 0 measured 54.0-54.5 -> 48.7 us on layer 1,
        // profiles/r5/hrow_mode1)
        if (MODE == 0 && r == 2 && hd) vm_wait<0>();
      } else {
        if (r == 0) {
          if (sig > 0) {
            if (epi_prev) vm_wait<ST>();
            else vm_wait<0>();
            bar_lds();
          }
        } else {
          if (hd && !(MODE >= 1 && r == 2)) vm_wait<HH>();
          else vm_wait<0>();
          bar_lds();
          if (MODE >= 1 && r == 2 && hd) {
            load_coef(cbD, hgrp);
            xform(buf ^ 1);
          }
        }
        if (r < 2) issue_w(n0, cl, r + 1, (sb + r + 1) % 2);
        else if (hd) issue_w(n0n, cbn, 0, (sb + 3) % 2);
      }
      if (r < 2 && hd) {
#pragma unroll
        for (int q = 0; q < HH; ++q) issue_h(cbD, buf ^ 1, r * HH + q);
      }
    };
    // fragments of tap t (both 32-deep halves) into register set u
    bf16x8 fa[2][2][TM], fb[2][2][TN];
    auto rd = [&](int u, int t) __attribute__((always_inline)) {
      const int r = t / 3, j = t % 3;
      const char* bs = smem + 2 * HBYTES + (STAT ? r : (sb + r) % 2) * WSLOT + j * BN * 128;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) fb[u][kk][tn] = *(const bf16x8*)(bs + bfo[kk][tn]);
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
          fa[u][kk][tm] = *(const bf16x8*)(hb + (aoff[t][tm] ^ (kk << 6)));
      }
    };
    row_start(0);
    rd(0, 0);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int u = t & 1;
      if (t + 1 < 9) {
        if ((t + 1) % 3 == 0) row_start((t + 1) / 3);
        rd(u ^ 1, t + 1);
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
          for (int tn = 0; tn < TN; ++tn)
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[u][kk][tn], fa[u][kk][tm],
                                                                 acc[tm][tn], 0, 0, 0);
      if (t + 1 < 9) {
        // the next tap's reads one per MFMA gap of this tap (left to itself the scheduler
        // issued each read right before its consumer with lgkmcnt(1) waits: LDS latency exposed)
        constexpr int NR = 2 * (TM + TN), NM = 2 * TM * TN;
        static_assert(NR <= NM, "reads fit the MFMA gaps");
#pragma unroll
        for (int x = 0; x < NR; ++x) {
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
        }
        __builtin_amdgcn_sched_group_barrier(0x008, NM - NR, 0);
      }
    }
    if (last_sl) {
      epi_lean<BM, BN, WM, NW, PERM>(acc, rsum, rsq, STATS, e, m0, n0, BM);
      if (STATS) {
        const int gcur = m0 / e.group_rows;
        if (!hd || n0n != n0 || m0n / e.group_rows != gcur)
          epi_flush<BM, BN, WM, NW, PERM>(rsum, rsq, (float*)(smem + buf * HBYTES), e, gcur,
                                          n0);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (hd) advance_d();
    m0 = m0n;
    n0 = n0n;
    sb = (sb + 3) % 2;
    if (last_sl) {
      cl = 0;
      ++k;
    } else {
      ++cl;
    }
  }
}

template <int BM, int BN, int NW>
int hrow_lds_bytes(const HconvGeom& g, bool stat) {
  const int hbytes = ((g.HPIX + 7) >> 3) * 8 * 128;
  constexpr int WM = BM / 64;   // (epilogue staging needs 2 * WM * BN floats of a halo buffer)
  if (hbytes < 2 * WM * BN * 4) return 1 << 30;
  return 2 * hbytes + (stat ? 3 : 2) * 3 * BN * 128;
}

template <int BM, int BN, int WM, int NW, int HRC, bool STAT, int MODE>
void launch_hrow_k(const bf16* src, const bf16* wt, const HconvGeom& g, const EpiParams& e,
                   const HconvPro& pro, int grid, int bytes, hipStream_t st) {
  static bool attr[2] = {false, false};
  const bool stats = e.stats != nullptr;
  if (!attr[stats]) {
    (void)hipFuncSetAttribute(
        stats ? (const void*)hrow_kernel<BM, BN, WM, NW, HRC, true, STAT, MODE>
              : (const void*)hrow_kernel<BM, BN, WM, NW, HRC, false, STAT, MODE>,
        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr[stats] = true;
  }
  if (stats)
    hipLaunchKernelGGL((hrow_kernel<BM, BN, WM, NW, HRC, true, STAT, MODE>), dim3(grid),
                       dim3(64 * NW), bytes, st, src, wt, g, e, pro);
  else
    hipLaunchKernelGGL((hrow_kernel<BM, BN, WM, NW, HRC, false, STAT, MODE>), dim3(grid),
                       dim3(64 * NW), bytes, st, src, wt, g, e, pro);
}

// 8 waves (two per SIMD), wave tiles 64 rows x 32 channels
template <int BM, int BN, int WM, int NW>
int launch_hrow(const bf16* src, const bf16* wt, const HconvGeom& g, const EpiParams& e,
                const HconvPro& pro, int grid, hipStream_t st) {
  const bool stat = g.C == 64 && g.K == BN;
  int bytes = hrow_lds_bytes<BM, BN, NW>(g, stat);
  if (bytes > 160 * 1024) return 0;
  // MODE 1: the coefficient table when it fits beside the tile and a block's tile range touches
  // at most two input statistics groups (N-tile-major ranges of <= one group's rows)
  HconvPro pr = pro;
  if (pro.mode == 1) {
    const int ntiles = (g.N * g.P * g.Q / BM) * (g.K / BN);
    const int per = (ntiles + grid - 1) / grid;
    const int grp_rows = pro.stats ? pro.group_imgs * g.P * g.Q : g.N * g.P * g.Q;
    if (bytes + 2 * g.C * 8 <= 160 * 1024 && per * BM <= grp_rows) {
      pr.coef_tab = 1;
      bytes += 2 * g.C * 8;
    }
  }
  // halo pieces of wave 0 (the most): 8 covers the ResNet layer1 / layer2 scoring tiles (6);
  // larger halos spill at 2 waves per SIMD -- not instantiated
  const int hr = ((g.HPIX + 7) / 8 + NW - 1) / NW;
  if (hr > 8) return 0;
  const int hrc = 8;
#define HR_CASE(H_)                                                                             \
  if (hrc == H_) {                                                                              \
    if (stat) {                                                                                 \
      if (pr.coef_tab) launch_hrow_k<BM, BN, WM, NW, H_, true, 2>(src, wt, g, e, pr, grid, bytes, st); \
      else if (pro.mode == 1) launch_hrow_k<BM, BN, WM, NW, H_, true, 1>(src, wt, g, e, pr, grid, bytes, st); \
      else launch_hrow_k<BM, BN, WM, NW, H_, true, 0>(src, wt, g, e, pr, grid, bytes, st);    \
    } else {                                                                                    \
      if (pr.coef_tab) launch_hrow_k<BM, BN, WM, NW, H_, false, 2>(src, wt, g, e, pr, grid, bytes, st); \
      else if (pro.mode == 1) launch_hrow_k<BM, BN, WM, NW, H_, false, 1>(src, wt, g, e, pr, grid, bytes, st); \
      else launch_hrow_k<BM, BN, WM, NW, H_, false, 0>(src, wt, g, e, pr, grid, bytes, st);   \
    }                                                                                           \
    return 1;                                                                                   \
  }
  HR_CASE(8)
#undef HR_CASE
  return 0;
}

// LDS of the persistent kernel: two halo buffers (each also the epilogue's staging area, so it
// must hold Smem::RED_BYTES), the weight ring, the DMA sink (1 KB per wave), and (MODE 1) the
// BN table of G x C scale / shift pairs
template <int BM, int BN, int NW>
int persist_lds_bytes(const HconvGeom& g, const HconvPro& pro) {
  const int ppx = 8 * NW;
  const int hbytes = ((g.HPIX + ppx - 1) / ppx) * ppx * 128;
  if (hbytes < Smem<BM, BN>::RED_BYTES) return 1 << 30;
  const int groups = pro.mode == 1 ? (pro.stats ? g.N / pro.group_imgs : 1) : 0;
  return 2 * hbytes + PSLOT * BN * 128 + NW * 1024 + groups * g.C * 8;
}

template <int BM, int BN, int WM, int NW, int HRC, int MODE>
void launch_persist_k(const bf16* src, const bf16* wt, const HconvGeom& g, const EpiParams& e,
                      const HconvPro& pro, int grid, int bytes, hipStream_t st) {
  static bool attr[2] = {false, false};
  const bool stats = e.stats != nullptr;
  if (!attr[stats]) {
    (void)hipFuncSetAttribute(
        stats ? (const void*)hconv_persist_kernel<BM, BN, WM, NW, 2, HRC, true, MODE>
              : (const void*)hconv_persist_kernel<BM, BN, WM, NW, 2, HRC, false, MODE>,
        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr[stats] = true;
  }
  if (stats)
    hipLaunchKernelGGL((hconv_persist_kernel<BM, BN, WM, NW, 2, HRC, true, MODE>), dim3(grid),
                       dim3(64 * NW), bytes, st, src, wt, g, e, pro);
  else
    hipLaunchKernelGGL((hconv_persist_kernel<BM, BN, WM, NW, 2, HRC, false, MODE>), dim3(grid),
                       dim3(64 * NW), bytes, st, src, wt, g, e, pro);
}

template <int BM, int BN, int WM, int NW, int HRC>
void launch_persist_m(const bf16* src, const bf16* wt, const HconvGeom& g, const EpiParams& e,
                      const HconvPro& pro, int grid, int bytes, hipStream_t st) {
  if (pro.mode == 1)
    launch_persist_k<BM, BN, WM, NW, HRC, 1>(src, wt, g, e, pro, grid, bytes, st);
  else
    launch_persist_k<BM, BN, WM, NW, HRC, 0>(src, wt, g, e, pro, grid, bytes, st);
}

// one block per CU of the grid; the halo piece capacity (8, 12 or 16 per wave) is the smallest
// that holds the tile's halo, so carrying taps issue few pieces into the sink
template <int BM, int BN, int WM, int NW>
int launch_persist_w(const bf16* src, const bf16* wt, const HconvGeom& g, const EpiParams& e,
                     const HconvPro& pro, int grid, hipStream_t st) {
  const int bytes = persist_lds_bytes<BM, BN, NW>(g, pro);
  if (bytes > 160 * 1024) return 0;
  const int hr = (g.HPIX + 8 * NW - 1) / (8 * NW);
  if (hr <= 8)
    launch_persist_m<BM, BN, WM, NW, 8>(src, wt, g, e, pro, grid, bytes, st);
  else if (hr <= 12)
    launch_persist_m<BM, BN, WM, NW, 12>(src, wt, g, e, pro, grid, bytes, st);
  else if (hr <= 16)
    launch_persist_m<BM, BN, WM, NW, 16>(src, wt, g, e, pro, grid, bytes, st);
  else
    return 0;
  return 1;
}

// WM4 / WM8: wave rows of the 4- and 8-wave blocks (MERCURY_HCONV_PERSIST_WAVES picks, 0 = none)
int g_persist_grid = 0;      // 0: half the CUs
int g_persist_waves = 8;     // 8 or 4
int g_persist_wm8 = 0;       // 8-wave wave-row count override (0: the tile's default WM8)

// WM8B: an alternative 8-wave layout of the same tile, selected by g_persist_wm8 == WM8B.  For
// 128 x 64 the default 8 x 1 wave grid gives every wave a 16 x 64 tile (1.25 KB of fragment
// reads per MFMA, each wave reading the whole weight tile); 4 x 2 gives 32 x 32 (1 KB per MFMA)
template <int BM, int BN, int WM4, int WM8, int WM8B = 0>
int launch_persist(const bf16* src, const bf16* wt, const HconvGeom& g, const EpiParams& e,
                   const HconvPro& pro, hipStream_t st) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
  }
  // blocks: half the CUs by default -- the scoring convs run beside the training stream, and a
  // grid on every CU (143 KB of LDS each) locks the training kernels out for its whole length.
  // Measured, ResNet-18 step (bench.py, same box): 256 blocks 1.653 ms, 192 1.590, 160 1.550,
  // 128 1.525, 96 1.720, 64 2.037; per-tile kernels 1.607.  hconv_configure() overrides (the
  // engine's EngineOptions.hconv_persist_grid / _waves).
  // 8 waves (two per SIMD: one wave's waits, barriers and DMA issue overlap the other's MFMAs)
  // where the tile has an 8-wave layout; measured 1.513 vs 1.521 and 1.534 vs 1.549 ms/step
  // (two same-box A/Bs), layer2 alone 33.4 vs 35.4 us
  int gmax = g.PGRID > 0 ? g.PGRID : (g_persist_grid > 0 ? g_persist_grid : cus / 2);
  if (gmax > cus) gmax = cus;
  const int waves = g_persist_waves;
  const int ntiles = (g.N * g.P * g.Q / (g.IMG * g.TR * g.Q)) * (g.K / BN);
  const int grid = ntiles < gmax ? ntiles : gmax;
  if constexpr (WM8 > 0) {
    if constexpr (WM8B > 0) {
      if (waves == 8 && g_persist_wm8 == WM8B)
        return launch_persist_w<BM, BN, WM8B, 8>(src, wt, g, e, pro, grid, st);
    }
    if (waves == 8) return launch_persist_w<BM, BN, WM8, 8>(src, wt, g, e, pro, grid, st);
  }
  return launch_persist_w<BM, BN, WM4, 4>(src, wt, g, e, pro, grid, st);
}

template <int BM, int BN, int WM>
void launch_one(const bf16* src, const bf16* wt, const HconvGeom& g, const EpiParams& e,
                dim3 grid, hipStream_t st) {
  const int hbytes = ((g.HPIX + 31) >> 5) * 32 * 128;
  const int nh = g.chunks_per_split > 1 ? 2 : 1;
  const int main_bytes = nh * hbytes + NSLOT * BN * 128 + 4096;
  const int red = Smem<BM, BN>::RED_BYTES;
  const int bytes = main_bytes > red ? main_bytes : red;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)hconv_kernel<BM, BN, WM>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL((hconv_kernel<BM, BN, WM>), grid, dim3(NT), bytes, st, src, wt, g, e);
}

}  // namespace

int hconv_read_stamps(unsigned long long* host, int n) {
#ifdef MERCURY_STAMPS
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 12 * n) ==
         hipSuccess;
#else
  (void)host;
  (void)n;
  return 0;
#endif
}

void hconv_configure(int grid, int waves, int wm8) {
  g_persist_grid = grid > 0 ? grid : 0;
  g_persist_waves = waves == 4 ? 4 : 8;
  g_persist_wm8 = wm8 > 0 ? wm8 : 0;
}

int hconv_lds_bytes(const HconvGeom& g, int bm, int bn, int splits_gt1) {
  const int hbytes = ((g.HPIX + 31) >> 5) * 32 * 128;
  const int main_bytes = (splits_gt1 ? 2 : 1) * hbytes + NSLOT * bn * 128 + 4096;
  const int red = 16 * bn * 4 + bm * (bn + 8) * 2;
  return main_bytes > red ? main_bytes : red;
}

int hconv_launch(const bf16* src, const bf16* wt, const HconvGeom& g_in, const EpiParams& e_in,
                 const HconvPro& pro, int bm, int bn, int splits, hipStream_t st) {
  HconvGeom g = g_in;
  g.zero = conv_zero_page();
  EpiParams e = e_in;
  const int M = g.N * g.P * g.Q;
  const int gx = ((M + bm - 1) / bm) * ((g.K + bn - 1) / bn);
  const int nchunks = g.C >> 6;
  if (splits <= 0 && g.SWA != 0) return 0;       // persistent / row-step halo images: SWA 0
  // rows per tile: bm, or (persistent kernel only) fewer whole image rows padded to bm
  const int vr = g.IMG * g.TR * g.Q;
  if (vr > bm || vr <= 0 || (vr != bm && splits != 0)) return 0;
  if (splits < 0) {
    // row-step persistent kernel (splits -1; 8 waves, 256 x 64 tiles): plain stride-1 input,
    // whole tiles, ghost-BN groups made of whole tiles
    const bool ok = (pro.mode == 0 || pro.mode == 1) &&
                    e.bias == nullptr && !e.accumulate &&
                    e.bw_sums == nullptr && g.stride == 1 && g.R == 3 && M % bm == 0 &&
                    g.K % bn == 0 && (e.stats == nullptr || e.group_rows % bm == 0);
    if (!ok) return 0;
    // the kernel's address packing: a halo slot holds its byte offset within the tile's
    // images in 26 bits and its halo row (63 = padding) above them, the tile base is an int and
    // the buffer resource's byte count an unsigned (a plan override outside this contract
    // falls back to the caller's other kernels instead of reading clamped addresses)
    const long long tile_bytes = (long long)g.IMG * g.H * g.W * g.C * 2;
    const long long in_bytes = (long long)g.N * g.H * g.W * g.C * 2;
    if (g.HT >= 63 || tile_bytes >= (1ll << 26) || in_bytes >= (1ll << 31)) return 0;
    static int cus = 0;
    if (!cus) {
      int dev = 0;
      (void)hipGetDevice(&dev);
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
          cus <= 0)
        cus = 256;
    }
    int gmax = g_persist_grid > 0 ? g_persist_grid : cus / 2;
    if (gmax > cus) gmax = cus;
    const int grid = gx < gmax ? gx : gmax;
    e.slab = nullptr;
    if (bm == 256 && bn == 64) return launch_hrow<256, 64, 4, 8>(src, wt, g, e, pro, grid, st);
    return 0;
  }
  const bool persist = splits == 0;
  splits = splits < 1 ? 1 : (splits > nchunks ? nchunks : splits);
  g.chunks_per_split = (nchunks + splits - 1) / splits;
  int gy = (nchunks + g.chunks_per_split - 1) / g.chunks_per_split;
  if (gx > 1024) gy = 1, g.chunks_per_split = nchunks;    // tile counters: SEM_INTS
  if (gy == 1) e.slab = nullptr;
  if (((g.HPIX + 31) >> 5) > HRMAX || g.R != 3) return 0;
  if (persist) {
    // persistent plan (splits == 0): plain whole tiles only, else the per-tile kernel below
    const bool ok = (pro.mode == 0 || pro.mode == 1) &&
                    e.bias == nullptr && !e.accumulate &&
                    e.bw_sums == nullptr && M % vr == 0 && g.K % bn == 0 &&
                    (e.stats == nullptr || e.group_rows % vr == 0);
#define HP_CASE(BM_, BN_, WM4_, WM8_, WM8B_)                                          \
  if (ok && bm == BM_ && bn == BN_ &&                                                  \
      launch_persist<BM_, BN_, WM4_, WM8_, WM8B_>(src, wt, g, e, pro, st))              \
    return 1;
    HP_CASE(256, 64, 4, 8, 0)
    HP_CASE(128, 64, 2, 8, 4)
    HP_CASE(64, 64, 1, 0, 0)
#undef HP_CASE
  }
  if (pro.mode != 0) return 0;      // the per-tile kernel stages plain input only
  const dim3 grid(gx, gy);
#define HC_CASE(BM_, BN_, WM_)                                  \
  if (bm == BM_ && bn == BN_) {                                 \
    launch_one<BM_, BN_, WM_>(src, wt, g, e, grid, st);         \
    return 1;                                                   \
  }
  HC_CASE(256, 64, 4)
  HC_CASE(128, 64, 2)
  HC_CASE(64, 64, 1)
  HC_CASE(256, 128, 4)
  HC_CASE(128, 128, 2)
  HC_CASE(64, 128, 1)
#undef HC_CASE
  return 0;
}
