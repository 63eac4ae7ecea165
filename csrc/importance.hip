// Importance-sampling data path on the GPU.
//
// pool_build  : the presample pool straight from the HBM-resident uint8 shard --
//               epoch shuffle (Feistel permutation, drop_last), RandomCrop(32, pad 4),
//               RandomHorizontalFlip, ToTensor, Normalize (`cifar10/data_loader.py:83-90`)
//               -> NHWC bf16 with channels padded to 8.  Replaces 352 PIL-augmented
//               images per step on the CPU.
// is_sample   : the whole `update_samples` tail (`pytorch_collab.py:106-117`) in one
//               workgroup: 10x EMA replay over the cumulative pool means (device-
//               resident EMAverage), p = (l + alpha*ema)/sum, inverse-CDF draws with
//               replacement (block-wide LDS prefix scan + binary search, Philox
//               uniforms), importance weights N*p[idx].
// gather      : the drawn samples' exact augmented views -> the next training batch.
// (the global importance table of Groupwise_Sampler lives in table.hip)
#include "common.h"
#include "kernels.h"

namespace {

// Which shard sample fills pool slot `slot` (epoch permutation, drop_last batches), and the
// global batch number gb that seeds its augmentation.
MA_DEV uint32_t pool_src(const PoolBuildArgs& a, int slot, int64_t& gb, int& t) {
  const int j = slot / a.batch;
  t = slot - j * a.batch;
  const int64_t pc = a.ctrl[0];
  const int per_pool = a.P / a.batch;
  const int nb = max(1, a.Ns / a.batch);
  gb = pc * per_pool + j;
  const uint32_t epoch = (uint32_t)(gb / nb);
  const int bi = (int)(gb % nb);
  // (% Ns only matters for a shard smaller than one batch: the batch cycles the shard)
  const uint32_t pos = (uint32_t)((bi * a.batch + t) % a.Ns);
  return a.shuffle ? permute_index(pos, (uint32_t)a.Ns, a.seed, epoch)
                   : (uint32_t)((gb * a.batch + t) % a.Ns);
}

// Pre-converted shard (non-image inputs, e.g. the speech VGG's 1x101x161 spectrograms, stored
// once as NHWC bf16 with channels padded to 8): the pool is a straight 16-byte-chunk gather.
MA_DEV void zero_slice(const PoolBuildArgs& a) {
  for (int j = blockIdx.x * 256 + threadIdx.x; j < a.nzero; j += gridDim.x * 256) a.zero[j] = 0.f;
}

__global__ __launch_bounds__(256) void pool_take_kernel(PoolBuildArgs a) {
  const int slot = blockIdx.x;
  if (a.zero) zero_slice(a);
  int64_t gb;
  int t;
  const uint32_t src = pool_src(a, slot, gb, t);
  if (threadIdx.x == 0) {
    a.pool_label[slot] = (int)a.labels[src];
    a.pool_index[slot] = (int)src;
  }
  const int npx = a.H * a.W;
  const u32x4* in = (const u32x4*)a.shard + (size_t)src * npx;
  u32x4* out = (u32x4*)a.pool + (size_t)slot * npx;
  for (int px = threadIdx.x; px < npx; px += 256) out[px] = in[px];
}

__global__ __launch_bounds__(256) void pool_build_kernel(PoolBuildArgs a) {
  const int slot = blockIdx.x;
  if (a.zero) zero_slice(a);
  int64_t gb;
  int t;
  const uint32_t src = pool_src(a, slot, gb, t);
  int dy = a.pad, dx = a.pad, flip = 0;
  if (a.augment) {
    const u32x4 r = philox4x32(u32x4{(uint32_t)gb, (uint32_t)(gb >> 32), (uint32_t)t, 0x5eedu},
                               a.seed, 0xA5A5A5A5u);
    dy = r.x % (2 * a.pad + 1);
    dx = r.y % (2 * a.pad + 1);
    flip = a.flip ? (r.z & 1) : 0;
  }
  if (threadIdx.x == 0) {
    a.pool_label[slot] = (int)a.labels[src];
    a.pool_index[slot] = (int)src;
  }
  const uint8_t* img = a.shard + (size_t)src * a.H * a.W * 3;
  bf16* out = a.pool + (size_t)slot * a.H * a.W * 8;
  const int npx = a.H * a.W;
  for (int px = threadIdx.x; px < npx; px += 256) {
    const int h = px / a.W, w = px - h * a.W;
    const int wc = flip ? (a.W - 1 - w) : w;
    const int hs = h + dy - a.pad, ws = wc + dx - a.pad;
    float v[3] = {0.f, 0.f, 0.f};
    if (hs >= 0 && ws >= 0 && hs < a.H && ws < a.W) {
      const uint8_t* p = img + ((size_t)hs * a.W + ws) * 3;
      v[0] = p[0];
      v[1] = p[1];
      v[2] = p[2];
    }
    bf16x8 o;
#pragma unroll
    for (int c = 0; c < 3; ++c) o[c] = f2bf((v[c] * (1.f / 255.f) - a.mean[c]) * a.inv_std[c]);
#pragma unroll
    for (int c = 3; c < 8; ++c) o[c] = f2bf(0.f);
    *(bf16x8*)(out + (size_t)px * 8) = o;
  }
}

constexpr int IS_T = 1024;
constexpr int MAX_GROUPS = 1024;  // pool batches per pool
constexpr int IS_LDS_MAX = 128 * 1024;   // dynamic LDS cap (static gsum[] rides on top)
constexpr int IS_W = IS_T / 64;          // waves per block

// Inclusive scan of one value per thread over the IS_T-thread block: a 64-lane shuffle scan per
// wave, the IS_W wave totals scanned by wave 0, added back -- two barriers (a Hillis-Steele scan
// over the block's LDS took 2 x log2(IS_T) = 20).  ``wt``: IS_W LDS slots of this call's own.
template <typename T>
MA_DEV T is_block_scan(T v, T* wt) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const T t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  if (lane == 63) wt[w] = v;
  __syncthreads();
  if (w == 0) {
    T t = lane < IS_W ? wt[lane] : T(0);
#pragma unroll
    for (int o = 1; o < IS_W; o <<= 1) {
      const T u = __shfl_up(t, o, 64);
      if (lane >= o) t += u;
    }
    if (lane < IS_W) wt[lane] = t;
  }
  __syncthreads();
  return w > 0 ? v + wt[w - 1] : v;
}

__global__ __launch_bounds__(IS_T) void is_sample_kernel(IsSampleArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* p = lds;                   // [P] probabilities, then CDF
  float* tsum = lds + a.P;          // [IS_T] per-thread segment sums (inclusive scan)
  float* red = tsum + IS_T;         // [64]
  const int tid = threadIdx.x;
  const int G = a.P / a.group;
  for (int i = tid; i < a.P; i += IS_T) p[i] = a.losses[i];
  __syncthreads();
  // group sums (over this rank's pool, or over every rank's pool when the gathered W x P
  // score matrix is given -- the global-EMA mode) -> cumulative means -> EMA replay
  // (10 updates for the reference pool)
  __shared__ float gsum[MAX_GROUPS];
  const float* src = a.gl ? a.gl : a.losses;
  const int rows = a.gl ? a.W : 1;
  for (int i = tid; i < G; i += IS_T) gsum[i] = 0.f;
  __syncthreads();
  for (int pr = tid; pr < rows * G; pr += IS_T) {
    const int r = pr / G, gi = pr - r * G;
    const float* q = src + (size_t)r * a.P + gi * a.group;
    float s = 0.f;
    for (int k = 0; k < a.group; ++k) s += q[k];
    atomicAdd(&gsum[gi], s);
  }
  __syncthreads();
  if (tid == 0) {
    float ema = a.ema[0];
    bool init = a.ema[1] != 0.f;
    double cs = 0.0;
    for (int gi = 0; gi < G; ++gi) {
      cs += gsum[gi];
      const float m = (float)(cs / (double)((gi + 1) * a.group * rows));
      if (!init) {
        ema = m;
        init = true;
      } else {
        ema = a.ema_alpha * ema + (1.f - a.ema_alpha) * m;
      }
    }
    a.ema[0] = ema;
    a.ema[1] = 1.f;
    red[32] = ema;
    red[33] = (float)(cs / (double)(a.P * rows));
    if (a.meters) {
      a.meters[3] = red[33];
      a.meters[4] = ema;
    }
  }
  __syncthreads();
  const float ema = red[32];
  // shifted weights and per-thread contiguous segment sums
  const int seg = (a.P + IS_T - 1) / IS_T;
  const int s0 = min(a.P, tid * seg), s1 = min(a.P, s0 + seg);
  float local = 0.f;
  for (int i = s0; i < s1; ++i) {
    const float v = a.importance ? (p[i] + a.alpha * ema) : 1.f;
    p[i] = v;
    local += v;
  }
  __shared__ float wt_p[IS_W], wt_d[IS_W], wt_e[IS_W];
  __shared__ int wt_c[IS_W];
  tsum[tid] = is_block_scan(local, wt_p);
  __syncthreads();
  const float total = tsum[IS_T - 1];
  const int64_t dc = a.ctrl[1];
  if (a.alias) {
    // Walker alias table built in PARALLEL in LDS (prob q[], alias al[]), then O(1) draws.
    // Sequential Vose pairs one light with one heavy at a time (a P-long dependent chain:
    // 70 us at P=320 on one lane).  The sweep it performs has a closed form (the PSA of
    // Huebschle-Schneider & Sanders): with the lights' exclusive deficit prefix D_i and the
    // heavies' exclusive excess prefix S_k,
    //   light i's alias  = heavy k, the smallest k with D_i <= S_{k+1};
    //   heavy k's prob   = 1 - (D_next - S_{k+1}), D_next = first light deficit prefix > S_{k+1},
    //   heavy k's alias  = heavy k+1 (it was topped up by the next heavy in the sweep),
    // so the build is three block scans + two binary searches per item.
    float* q = tsum + IS_T + 64;                 // [P] bucket probability
    int* al = (int*)(q + a.P);                   // [P] alias
    int* Lidx = al + a.P;                        // [P] light items in order
    int* Hidx = Lidx + a.P;                      // [P] heavy items in order
    float* Ld = (float*)(Hidx + a.P);            // [P] exclusive deficit prefix of lights
    float* Hs = Ld + a.P;                        // [P+1] exclusive excess prefix of heavies
    int* ccnt = (int*)(Hs + a.P + 1);            // [IS_T] light-count scan
    float* cdef = (float*)(ccnt + IS_T);         // [IS_T] deficit scan
    float* cexc = cdef + IS_T;                   // [IS_T] excess scan
    const float scale = (float)a.P / total;
    int lc = 0;
    float ld = 0.f, he = 0.f;
    for (int i = s0; i < s1; ++i) {
      const float v = p[i] * scale;
      q[i] = v;
      if (v < 1.f) {
        ++lc;
        ld += 1.f - v;
      } else {
        he += v - 1.f;
      }
    }
    ccnt[tid] = is_block_scan(lc, wt_c);
    cdef[tid] = is_block_scan(ld, wt_d);
    cexc[tid] = is_block_scan(he, wt_e);
    __syncthreads();
    {
      int li = tid > 0 ? ccnt[tid - 1] : 0, hi = s0 - li;
      float dd = tid > 0 ? cdef[tid - 1] : 0.f, ee = tid > 0 ? cexc[tid - 1] : 0.f;
      for (int i = s0; i < s1; ++i) {
        const float v = q[i];
        if (v < 1.f) {
          Lidx[li] = i;
          Ld[li++] = dd;
          dd += 1.f - v;
        } else {
          Hidx[hi] = i;
          Hs[hi++] = ee;
          ee += v - 1.f;
        }
      }
    }
    const int nl = ccnt[IS_T - 1], nh = a.P - nl;
    if (tid == 0) Hs[nh] = cexc[IS_T - 1];
    __syncthreads();
    const float dtot = cdef[IS_T - 1];
    for (int j = tid; j < nl; j += IS_T) {      // lights: who tops me up
      const float D = Ld[j];
      int lo = 0, hi = nh - 1;                   // smallest k with D <= Hs[k+1]
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (D <= Hs[mid + 1]) hi = mid;
        else lo = mid + 1;
      }
      al[Lidx[j]] = nh > 0 ? Hidx[lo] : Lidx[j];
      if (nh == 0) q[Lidx[j]] = 1.f;             // numerically all-light: uniform fallback
    }
    for (int k = tid; k < nh; k += IS_T) {      // heavies: what is left in my own bucket
      const float S1 = Hs[k + 1];
      int lo = 0, hi = nl;                       // first light with Ld > S1
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (Ld[mid] > S1) hi = mid;
        else lo = mid + 1;
      }
      const float Dn = lo < nl ? Ld[lo] : dtot;
      const float r = (k == nh - 1) ? 1.f : fminf(1.f, fmaxf(0.f, 1.f - (Dn - S1)));
      q[Hidx[k]] = r;
      al[Hidx[k]] = k + 1 < nh ? Hidx[k + 1] : Hidx[k];
    }
    __syncthreads();
    for (int d = tid; d < a.B; d += IS_T) {
      const u32x4 r = philox4x32(u32x4{(uint32_t)dc, (uint32_t)(dc >> 32), (uint32_t)d, 0xa11au},
                                 a.seed, 0x3C6EF372u);
      const int bin = min((int)(u01(r.x) * (float)a.P), a.P - 1);
      const int pick = u01(r.y) < q[bin] ? bin : al[bin];
      a.idx[d] = pick;
      a.w[d] = a.importance ? p[pick] / total * (float)a.P : 1.f;
    }
    __syncthreads();
    if (tid == 0) {
      a.ctrl[0] += 1;
      a.ctrl[1] += 1;
    }
    return;
  }
  float run = tid > 0 ? tsum[tid - 1] : 0.f;
  for (int i = s0; i < s1; ++i) {
    run += p[i];
    p[i] = run;  // unnormalised CDF
  }
  __syncthreads();
  for (int d = tid; d < a.B; d += IS_T) {
    const u32x4 r = philox4x32(u32x4{(uint32_t)dc, (uint32_t)(dc >> 32), (uint32_t)d, 0xd1a5u},
                               a.seed, 0x3C6EF372u);
    const float u = u01(r.x) * total;
    int lo = 0, hi = a.P - 1;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (p[mid] > u) hi = mid;
      else lo = mid + 1;
    }
    const float prev = lo > 0 ? p[lo - 1] : 0.f;
    a.idx[d] = lo;
    a.w[d] = a.importance ? (p[lo] - prev) / total * (float)a.P : 1.f;
  }
  __syncthreads();
  if (tid == 0) {
    a.ctrl[0] += 1;
    a.ctrl[1] += 1;
  }
}

__global__ __launch_bounds__(256) void gather_kernel(GatherArgs a) {
  const int b = blockIdx.y;
  const int s = a.idx[b];
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < a.chunks_per_img) {
    const u32x4 v = ((const u32x4*)a.pool)[(size_t)s * a.chunks_per_img + i];
    ((u32x4*)a.batch)[(size_t)b * a.chunks_per_img + i] = v;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    a.batch_label[b] = a.pool_label[s];
    if (a.batch_index) a.batch_index[b] = a.pool_index[s];
  }
}

}  // namespace

void pool_build_launch(const PoolBuildArgs& a, hipStream_t st) {
  if (a.prebuilt)
    hipLaunchKernelGGL(pool_take_kernel, dim3(a.P), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(pool_build_kernel, dim3(a.P), dim3(256), 0, st, a);
}

size_t is_sample_lds(int P, int alias) {
  return (size_t)(P + IS_T + 64) * sizeof(float) +
         (alias ? (6 * (size_t)P + 1 + 3 * IS_T) * 4 : 0);
}

void is_sample_launch(const IsSampleArgs& a, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)is_sample_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                        IS_LDS_MAX);
    attr = true;
  }
  hipLaunchKernelGGL(is_sample_kernel, dim3(1), dim3(IS_T), is_sample_lds(a.P, a.alias), st, a);
}

void gather_launch(const GatherArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(gather_kernel, dim3((a.chunks_per_img + 255) / 256, a.B), dim3(256), 0, st, a);
}
