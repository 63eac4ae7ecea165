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

__global__ __launch_bounds__(256) void pool_build_kernel(PoolBuildArgs a) {
  const int slot = blockIdx.x;
  const int j = slot / a.batch, t = slot - j * a.batch;
  const int64_t pc = a.ctrl[0];
  const int per_pool = a.P / a.batch;
  const int nb = max(1, a.Ns / a.batch);
  const int64_t gb = pc * per_pool + j;
  const uint32_t epoch = (uint32_t)(gb / nb);
  const int bi = (int)(gb % nb);
  const uint32_t pos = (uint32_t)(bi * a.batch + t);
  const uint32_t src = a.shuffle ? permute_index(pos, (uint32_t)a.Ns, a.seed, epoch)
                                 : (uint32_t)((gb * a.batch + t) % a.Ns);
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
constexpr int MAX_GROUPS = 256;   // pool batches per pool

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
  tsum[tid] = local;
  __syncthreads();
  for (int off = 1; off < IS_T; off <<= 1) {  // Hillis-Steele inclusive scan
    const float add = tid >= off ? tsum[tid - off] : 0.f;
    __syncthreads();
    tsum[tid] += add;
    __syncthreads();
  }
  const float total = tsum[IS_T - 1];
  const int64_t dc = a.ctrl[1];
  if (a.alias) {
    // Walker/Vose alias table in LDS (prob in q[], alias[]), then O(1) draws.
    float* q = tsum + IS_T + 64;                 // [P]
    int* al = (int*)(q + a.P);                   // [P]
    int* small = al + a.P;                       // [P]
    int* large = small + a.P;                    // [P]
    const float scale = (float)a.P / total;
    for (int i = tid; i < a.P; i += IS_T) {
      q[i] = p[i] * scale;
      al[i] = i;
    }
    __syncthreads();
    if (tid == 0) {
      int ns = 0, nl = 0;
      for (int i = 0; i < a.P; ++i) {
        if (q[i] < 1.f) small[ns++] = i;
        else large[nl++] = i;
      }
      while (ns > 0 && nl > 0) {
        const int s = small[--ns], l = large[--nl];
        al[s] = l;                               // q[s] stays as prob[s]
        q[l] = (q[l] + q[s]) - 1.f;
        if (q[l] < 1.f) small[ns++] = l;
        else large[nl++] = l;
      }
      while (nl > 0) q[large[--nl]] = 1.f;
      while (ns > 0) q[small[--ns]] = 1.f;       // numerical leftovers
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
  hipLaunchKernelGGL(pool_build_kernel, dim3(a.P), dim3(256), 0, st, a);
}

void is_sample_launch(const IsSampleArgs& a, hipStream_t st) {
  const size_t shm = (size_t)(a.P + IS_T + 64) * sizeof(float) + (a.alias ? 4 * (size_t)a.P * 4 : 0);
  hipLaunchKernelGGL(is_sample_kernel, dim3(1), dim3(IS_T), shm, st, a);
}

void gather_launch(const GatherArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(gather_kernel, dim3((a.chunks_per_img + 255) / 256, a.B), dim3(256), 0, st, a);
}
