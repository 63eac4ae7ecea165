// Narrow-input pointwise (1x1) convolution with the input's BatchNorm applied ONCE per element:
// the "expansion" convs -- ResNet-50's bottleneck conv3 (64 -> 256 at 56x56, 128 -> 512 at 28x28,
// `pytorch_model.py:44-49`) and MobileNetV2's expand convs -- read a narrow (K <= 128 channel)
// activation and write a 4-6x wider one, so they are bound by HBM, not MFMA.
//
// A block owns BM = 128 output rows and ALL output channels:
//   1. its A panel (128 rows x K <= 128 channels, <= 32 KB) lands in LDS by buffer LDS-DMA;
//   2. each thread normalises the chunks its own DMA brought, in place: a = act(bn(y)) from the
//      producer's per-group scale / shift (PRO), and writes the activation to ``keep`` once
//      (no N-tile redoes the transform: the block holds the panel for every N-tile);
//   3. it walks the N-tiles (BN = 64 channels) with the weight tile double-buffered in LDS (the
//      next one's DMA in flight under the current MFMAs) and a direct-from-register epilogue
//      (8-byte NHWC stores, ghost-BN statistics reduced by DPP rows and one LDS pass, one atomic
//      pair per channel per tile).
// The activation is read from HBM exactly once; the producer's separate bn_apply pass (read y,
// write a) disappears.  ~64 KB of LDS per block: two blocks per CU hide each other's DMA
// latency.  LDS image and fragment reads as in pgemm.hip (64-byte rows, chunk c of row r at
// c ^ ((r >> 1) & 3): conflict-free for ds_read_b128, bench/lds_swizzle_check.py).
#include "common.h"
#include "igemm.h"

namespace {

constexpr int PW_BM = 128;       // rows per block
constexpr int PW_BN = 64;        // output channels per N-tile
constexpr int PW_NT = 256;       // 4 waves, 2 (M) x 2 (N): 64 x 32 per wave
constexpr int PW_KMAX = 128;     // input channels held in the panel
constexpr unsigned PW_OOB = 0xFFFFFF00u;
// output staging tile [BM][BN] bf16: 128-byte rows, 16-byte chunk p of row r at slot p ^ (r & 7)
// (the 8-byte accumulator writes of 16 rows then hit 2-way at most, the 16-byte row reads none)
constexpr int PW_OBYTES = PW_BM * PW_BN * 2;
MA_DEV int pw_soff(int r, int c) {       // byte offset of (row r, channel c) in the staging tile
  return r * (PW_BN * 2) + (((c >> 3) ^ (r & 7)) << 4) + ((c & 7) << 1);
}

MA_DEV unsigned pw_lds_addr(const void* p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) char*)p;
}
MA_DEV __amdgpu_buffer_rsrc_t pw_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, bytes, 0x00020000);
}
MA_DEV void pw_dma16(__amdgpu_buffer_rsrc_t r, unsigned off, unsigned lds) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
               ::"v"(off), "s"(r), "s"(lds) : "memory");
}
template <int N>
MA_DEV void pw_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
MA_DEV void pw_bar_lds() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
MA_DEV float pw_row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  return v;
}
typedef uint32_t pw_u32x2 __attribute__((ext_vector_type(2)));

// 16-byte stores per thread of a staged [BM][BN] output tile: a row's BN * 2 = 128 bytes are 8
// consecutive lanes, so one wave instruction writes 8 whole 128-byte row segments (the
// direct-from-accumulator form wrote 16 rows x 32 bytes per instruction: these expansion convs
// are write-bound, 2 GB out per 0.5 GB in at ResNet-50's layer1)
constexpr int PW_ST = PW_BM * PW_BN * 2 / 16 / PW_NT;   // stores per thread per N-tile (4)
MA_DEV void pw_store_tile(const char* sO, __amdgpu_buffer_rsrc_t rs_o, const PgemmArgs& g,
                          int m0, int n0, int tid) {
#pragma unroll
  for (int i = 0; i < PW_ST; ++i) {
    const int c = tid + PW_NT * i;                   // 16-byte chunk of the tile
    const int r = c >> 3, piece = c & 7;             // (PW_BN * 2 / 16 = 8 chunks per row)
    const u32x4 v = *(const u32x4*)(sO + pw_soff(r, piece * 8));
    const int row = m0 + r, col = n0 + piece * 8;
    const bool ok = row < g.M && col < g.N;          // (N % 8 == 0: a chunk is whole or out)
    __builtin_amdgcn_raw_buffer_store_b128(
        v, rs_o, ok ? (unsigned)(((long long)row * g.ldo + col) * 2) : PW_OOB, 0, 0);
  }
}

// KB = 32-deep k-blocks of the panel (K <= 32 * KB); PRO: input prologue on
template <int KB, bool PRO, bool STATS>
__global__ __launch_bounds__(PW_NT, 2) void pwconv_kernel(PgemmArgs g, PgemmPro pro) {
  constexpr int BM = PW_BM, BN = PW_BN;
  constexpr int TM = 4, TN = 2;                      // 64 x 32 per wave
  constexpr int SA = KB * BM * 64;                   // A panel bytes
  constexpr int SBT = KB * BN * 64;                  // one weight tile
  // staged epilogue: a 16 KB tile area of its own for a shallow panel (KB <= 2: 64 -> 256 @56
  // 810 -> 644 us); deeper panels stage into the weight tile the MFMAs just finished (one more
  // barrier per N-tile): a separate area there cost the second block per CU (128 -> 512 @28
  // 479 -> 552 us with a padded 18 KB area)
  constexpr bool STAGE = true;
  constexpr bool OWN = KB <= 2 || SBT < PW_OBYTES;
  constexpr int PA = KB * (BM / 16) / 4;             // A pieces per wave (KB * 2)
  constexpr int PB = KB * (BN / 16) / 4;             // B pieces per wave per N-tile (KB)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sA = smem;
  char* sB = smem + SA;                              // [2][SBT]
  float* red = (float*)(smem + SA + 2 * SBT);        // [2 wave rows][2][BN]
  // output staging tile [BM][BN] bf16 (pw_soff layout): the accumulators land here (8 bytes per
  // lane) and leave as 16-byte row-contiguous stores (see the epilogue)
  char* sO = smem + SA + 2 * SBT + 2 * 2 * BN * 4;   // (OWN; else the weight tile, per N-tile)

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const int wm = w >> 1, wn = w & 1;
  const int m0 = blockIdx.x * BM;
  const int ntn = (g.N + BN - 1) / BN;
  const int K8 = g.K >> 3;
  const auto rs_a = pw_rsrc(g.a, g.a_bytes);
  const auto rs_b = pw_rsrc(g.b, g.b_bytes);
  const auto rs_o = pw_rsrc(g.out, g.out_bytes);
  const auto rs_k = pw_rsrc(pro.keep, pro.keep_bytes);
  const unsigned a_lds = pw_lds_addr(sA), b_lds = pw_lds_addr(sB);

  // DMA lane roles (16-row x 64-byte pieces): row lane >> 2, physical chunk lane & 3, logical lc
  const int prow = lane >> 2;
  const int lc = (lane & 3) ^ ((prow >> 1) & 3);
  // piece q of this wave: k-block q / (BM / 64), row block (q % (BM / 64)) * 4 + wu
  auto a_piece = [&](int q, int& kb, int& rb) {
    kb = q / (BM / 64);
    rb = (q % (BM / 64)) * 4 + wu;
  };
  auto issue_b = [&](int nt, int buf) {
#pragma unroll
    for (int q = 0; q < PB; ++q) {
      const int kb = q, rb = wu;                      // BN / 16 = 4 row blocks: one per wave
      const int n = nt * BN + rb * 16 + prow;
      const bool ok = n < g.N && kb * 4 + lc < K8;
      pw_dma16(rs_b, ok ? (unsigned)((n * g.K + kb * 32 + lc * 8) * 2) : PW_OOB,
               b_lds + buf * SBT + (kb * BN + rb * 16) * 64);
    }
  };

  // ---- 1. A panel + the first weight tile in flight
#pragma unroll
  for (int q = 0; q < PA; ++q) {
    int kb, rb;
    a_piece(q, kb, rb);
    const int m = m0 + rb * 16 + prow;
    const bool ok = m < g.M && kb * 4 + lc < K8;
    pw_dma16(rs_a, ok ? (unsigned)(((long long)m * g.K + kb * 32 + lc * 8) * 2) : PW_OOB,
             a_lds + (kb * BM + rb * 16) * 64);
  }
  issue_b(0, 0);
  pw_wait<PB>();                                     // this wave's A pieces landed
  // ---- 2. normalise the own chunks in place (+ keep)
  if constexpr (PRO) {
    const float lo = pro.act == 0 ? __builtin_nanf("") : 0.f;
    const float hi = pro.act == 2 ? 6.f : (pro.act == 0 ? __builtin_nanf("") : __builtin_huge_valf());
    const int g0 = m0 / pro.group_rows, bnd = (g0 + 1) * pro.group_rows;
#pragma unroll
    for (int q = 0; q < PA; ++q) {
      int kb, rb;
      a_piece(q, kb, rb);
      const int m = m0 + rb * 16 + prow;
      const int ch = kb * 32 + lc * 8;
      if (ch >= g.K) continue;                       // zero-filled padding chunk
      const int gq = m >= bnd && g0 + 1 < pro.G ? g0 + 1 : g0;
      const float* cs = pro.coef + (size_t)gq * 2 * g.K + ch;
      const f32x4 c0 = *(const f32x4*)cs, c1 = *(const f32x4*)(cs + 4);
      const f32x4 h0 = *(const f32x4*)(cs + g.K), h1 = *(const f32x4*)(cs + g.K + 4);
      u32x4* ap = (u32x4*)(sA + (kb * BM + rb * 16) * 64 + lane * 16);
      const bf16x8 y = __builtin_bit_cast(bf16x8, *ap);
      bf16x8 o;
#pragma unroll
      for (int k = 0; k < 8; ++k)
        o[k] = f2bf(fminf(fmaxf(bf2f(y[k]) * (k < 4 ? c0[k] : c1[k - 4]) + (k < 4 ? h0[k] : h1[k - 4]), lo), hi));
      const u32x4 ov = __builtin_bit_cast(u32x4, o);
      *ap = ov;
      if (pro.keep)
        __builtin_amdgcn_raw_buffer_store_b128(
            ov, rs_k, m < g.M ? (unsigned)(((long long)m * g.K + ch) * 2) : PW_OOB, 0, 0);
    }
  }
  pw_wait<0>();
  pw_bar_lds();

  // ---- 3. N-tiles: weight tile nt + 1 in flight under tile nt's MFMAs
  const int fl = (lane & 15) * 64 + 16 * ((lane >> 4) ^ ((lane >> 1) & 3));
  const int rbase = m0 + wm * 64 + (lane & 15);
  int gs = 0, bnd = 0x7fffffff;
  if constexpr (STATS) {
    gs = m0 / g.group_rows;
    bnd = (gs + 1) * g.group_rows;
  }
  const bool straddle = STATS && bnd < m0 + BM && bnd < g.M;
  for (int nt = 0; nt < ntn; ++nt) {
    const int buf = nt & 1;
    if (nt + 1 < ntn) issue_b(nt + 1, buf ^ 1);
    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      bf16x8 fa[TM], fb[TN];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
        fa[tm] = *(const bf16x8*)(sA + (kb * BM + wm * 64 + tm * 16) * 64 + fl);
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
        fb[tn] = *(const bf16x8*)(sB + buf * SBT + (kb * BN + wn * 32 + tn * 16) * 64 + fl);
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[tn], fa[tm], acc[tm][tn], 0, 0, 0);
    }
    // epilogue: the tile through LDS (row-contiguous 16-byte stores) + statistics
    char* sOt = OWN ? sO : sB + buf * SBT;
    if constexpr (!OWN) pw_bar_lds();               // every wave's reads of the weight tile done
    const int cbase = nt * BN + wn * 32 + 4 * (lane >> 4);
    float s[TN][4], ss[TN][4], s2[TN][4], ss2[TN][4];
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
#pragma unroll
      for (int j = 0; j < 4; ++j) s[tn][j] = ss[tn][j] = s2[tn][j] = ss2[tn][j] = 0.f;
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int col = cbase + tn * 16;
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const int row = rbase + tm * 16;
        bf16x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = f2bf(acc[tm][tn][j]);
        if constexpr (STAGE) {
          // (tile-local row / column of this lane's 4 channels)
          *(pw_u32x2*)(sOt + pw_soff(row - m0, col - nt * BN)) = __builtin_bit_cast(pw_u32x2, o);
        } else {
          const bool ok = row < g.M && col < g.N;
          __builtin_amdgcn_raw_buffer_store_b64(
              __builtin_bit_cast(pw_u32x2, o), rs_o,
              ok ? (unsigned)(((long long)row * g.ldo + col) * 2) : PW_OOB, 0, 0);
        }
        if constexpr (STATS) {
          const float mk = row < g.M ? 1.f : 0.f;
          const float m1 = row < bnd ? mk : 0.f, m2 = mk - m1;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float f = bf2f(o[j]);
            s[tn][j] += f * m1;
            ss[tn][j] += f * f * m1;
            s2[tn][j] += f * m2;
            ss2[tn][j] += f * f * m2;
          }
        }
      }
    }
    if constexpr (STATS) {
      for (int part = 0; part < (straddle ? 2 : 1); ++part) {
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float a = pw_row16_sum(part ? s2[tn][j] : s[tn][j]);
            const float b = pw_row16_sum(part ? ss2[tn][j] : ss[tn][j]);
            if ((lane & 15) == 0) {
              const int cl = wn * 32 + tn * 16 + 4 * (lane >> 4) + j;
              red[(wm * 2) * BN + cl] = a;
              red[(wm * 2 + 1) * BN + cl] = b;
            }
          }
        }
        pw_bar_lds();
        if (tid < BN && nt * BN + tid < g.N) {
          float* dst = MA_SPREAD(g.stats + (size_t)(gs + part) * 2 * g.stats_ld + nt * BN + tid);
          atomicAdd(dst, red[tid] + red[2 * BN + tid]);
          atomicAdd(dst + g.stats_ld, red[BN + tid] + red[3 * BN + tid]);
        }
        if (STAGE && part == 0) pw_store_tile(sOt, rs_o, g, m0, nt * BN, tid);
        pw_bar_lds();
      }
    } else if constexpr (STAGE) {
      pw_bar_lds();                                  // the staging tile is complete
      pw_store_tile(sOt, rs_o, g, m0, nt * BN, tid);
    }
    // weight tile nt + 1 landed -- a COUNTED wait: the PW_ST stores of this tile (and wave 0's
    // statistics atomics) are younger than that DMA and stay in flight under the next tile's
    // MFMAs (vmcnt retires in issue order).  A vmcnt(0) here waited for every store's
    // acknowledgement once per N-tile: four store round trips per 128-row block at 2 blocks per
    // CU left these HBM-bound expansion convs at ~3.1 TB/s
    if (nt + 1 < ntn) {
      constexpr int NS = STAGE ? PW_ST : TM * TN;    // this thread's output stores of the tile
      if (STATS && wu == 0) {
        if (straddle) pw_wait<NS + 4>();
        else pw_wait<NS + 2>();
      } else {
        pw_wait<NS>();
      }
    }
    pw_bar_lds();
  }
}

template <int KB, bool PRO, bool STATS>
void pw_launch(const PgemmArgs& g, const PgemmPro& pro, hipStream_t st) {
  constexpr int SBT = KB * PW_BN * 64;
  constexpr int bytes = KB * PW_BM * 64 + 2 * SBT + 2 * 2 * PW_BN * 4 +
                        ((KB <= 2 || SBT < PW_OBYTES) ? PW_OBYTES : 0);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)pwconv_kernel<KB, PRO, STATS>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    attr = true;
  }
  hipLaunchKernelGGL((pwconv_kernel<KB, PRO, STATS>), dim3((g.M + PW_BM - 1) / PW_BM), dim3(PW_NT),
                     bytes, st, g, pro);
}

template <int KB>
void pw_launch_kb(const PgemmArgs& g, const PgemmPro& pro, hipStream_t st) {
  const bool stats = g.stats != nullptr;
  if (pro.mode == 1) {
    if (stats) pw_launch<KB, true, true>(g, pro, st);
    else pw_launch<KB, true, false>(g, pro, st);
  } else {
    if (stats) pw_launch<KB, false, true>(g, pro, st);
    else pw_launch<KB, false, false>(g, pro, st);
  }
}

__global__ __launch_bounds__(256) void pw_coef_kernel(PgemmPro p, int K) {
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

}  // namespace

// returns 0 when unsupported: K <= 128 input channels, stride 1, plain or mode-1 prologue,
// statistics groups of >= 128 rows (a block straddles at most one group edge)
int pwconv_launch(const PgemmArgs& g, hipStream_t st, const PgemmPro* pro_in) {
  PgemmPro pro{};
  if (pro_in) pro = *pro_in;
  if (g.K % 8 || g.N % 8 || g.K > PW_KMAX || g.stride != 1 || g.M <= 0) return 0;
  if (g.stats && g.group_rows < PW_BM) return 0;
  if (pro.mode == 2) return 0;
  if (pro.mode == 1) {
    if (!pro.coef || pro.G < 1 || pro.group_rows < PW_BM) return 0;
    hipLaunchKernelGGL(pw_coef_kernel, dim3((pro.G * g.K + 255) / 256), dim3(256), 0, st, pro, g.K);
  }
  switch ((g.K + 31) / 32) {
    case 1: pw_launch_kb<1>(g, pro, st); return 1;
    case 2: pw_launch_kb<2>(g, pro, st); return 1;
    case 3: pw_launch_kb<3>(g, pro, st); return 1;
    case 4: pw_launch_kb<4>(g, pro, st); return 1;
    default: return 0;
  }
}
