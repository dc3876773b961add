// Device-side data path: the synthetic phantom generator, the
// reference's ModalitySpecificNormalize (src/data/transforms.py:362-404) and
// Resize (transforms.py:215-250, scipy.ndimage.zoom order 1 / labels order 0)
// as HIP kernels, so a training batch never touches the host.
// oracle/data_oracle.py restates each one; tests/golden/transforms.npz pins the
// normalize / resize restatement to the reference's own transforms.
//
//   modality_normalize  CT: clip to the window, scale to [0, 1] (float32 math,
//                       bit-identical to the reference's numpy); PET: divide by
//                       the volume max (if > 0); MRI/US: z-score with fp64
//                       statistics (ddof 0, std + 1e-8).  Reductions are
//                       two-level and fixed-order.
//   resize_linear       per-axis corner-aligned linear interpolation in fp64,
//                       evaluated axis by axis (z, then y, then x) like the
//                       restatement; neighbours past the end carry weight 0
//   resize_nearest      labels (int64 or uint8): nearest input index, ties up
//   phantom             labels from host-drawn ellipsoids (fp64 tests in class
//                       order), intensities = class mean + std * N with N from a
//                       SplitMix64 counter stream through Box-Muller (fp64)
#include "mmseg_common.h"

namespace {

constexpr int NB = 256;           // first-level reduction blocks

__global__ void ct_window_kernel(float* __restrict__ x, long long V, float lo, float hi, float width) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < V; i += (long long)gridDim.x * blockDim.x) {
    float v = x[i];
    v = v < lo ? lo : (v > hi ? hi : v);
    x[i] = __fdiv_rn(__fsub_rn(v, lo), width);
  }
}

__device__ __forceinline__ double block_sum_d(double v, double* red) {
  v = wave_sum_d(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) red[wave] = v;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x == 0)
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
  return t;   // valid in thread 0
}

// per-block partial max (PET) / sum (z-score pass 1) / sum of squared deviations (pass 2)
__global__ __launch_bounds__(256) void stat_partial_kernel(const float* __restrict__ x, long long V, int what,
                                                           const double* __restrict__ stats,
                                                           double* __restrict__ part) {
  __shared__ double red[4];
  const long long per = (V + gridDim.x - 1) / gridDim.x;
  const long long b0 = (long long)blockIdx.x * per, b1 = b0 + per < V ? b0 + per : V;
  double acc = what == 0 ? -1.0e300 : 0.0;
  const double mean = what == 2 ? stats[0] : 0.0;
  for (long long i = b0 + threadIdx.x; i < b1; i += blockDim.x) {
    const double v = (double)x[i];
    if (what == 0) acc = v > acc ? v : acc;
    else if (what == 1) acc += v;
    else acc += (v - mean) * (v - mean);
  }
  if (what == 0) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double t = __shfl_xor(acc, o, 64);
      acc = t > acc ? t : acc;
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) red[wave] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
      double m = red[0];
      for (int w = 1; w < 4; ++w) m = red[w] > m ? red[w] : m;
      part[blockIdx.x] = m;
    }
    return;
  }
  const double t = block_sum_d(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

// stats[0] = max | mean, stats[1] = std + 1e-8 (what 2) from the partials, in block order
__global__ void stat_final_kernel(const double* __restrict__ part, int nb, int what, long long V,
                                  double* __restrict__ stats) {
  if (threadIdx.x != 0) return;
  double a = what == 0 ? part[0] : 0.0;
  for (int b = (what == 0 ? 1 : 0); b < nb; ++b) a = what == 0 ? (part[b] > a ? part[b] : a) : a + part[b];
  if (what == 0) stats[0] = a;
  else if (what == 1) stats[0] = a / (double)V;
  else stats[1] = sqrt(a / (double)V) + 1e-8;
}

// PET: x /= max (if max > 0); z-score: x = (x - (float)mean) / (float)std
__global__ void scale_kernel(float* __restrict__ x, long long V, int what, const double* __restrict__ stats) {
  if (what == 0) {
    const double m = stats[0];
    if (!(m > 0.0)) return;
    const float mf = (float)m;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < V; i += (long long)gridDim.x * blockDim.x)
      x[i] = __fdiv_rn(x[i], mf);
    return;
  }
  const float mean = (float)stats[0], sd = (float)stats[1];
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < V; i += (long long)gridDim.x * blockDim.x)
    x[i] = __fdiv_rn(__fsub_rn(x[i], mean), sd);
}

// ------------------------------------------------------------------ resize
struct AxisMap {
  int i0, i1v;     // first neighbour, second neighbour (clamped)
  double w0, w1;   // weights (w1 = 0 past the end)
};

__device__ __forceinline__ AxisMap axis_map(int o, int n_in, int n_out) {
  AxisMap m;
  const double z = n_out > 1 ? (double)(n_in - 1) / (double)(n_out - 1) : 0.0;
  const double x = __dmul_rn((double)o, z);
  const double fl = floor(x);
  m.i0 = (int)fl;
  const double f = __dsub_rn(x, fl);
  const int i1 = m.i0 + 1;
  m.i1v = i1 < n_in ? i1 : n_in - 1;
  m.w0 = __dsub_rn(1.0, f);
  m.w1 = i1 < n_in ? f : 0.0;
  if (m.i0 > n_in - 1) m.i0 = n_in - 1;
  return m;
}

__device__ __forceinline__ double lerp2(double a, double b, double w0, double w1) {
  return __dadd_rn(__dmul_rn(a, w0), __dmul_rn(b, w1));
}

__global__ void resize_linear_kernel(const float* __restrict__ src, int C, int D, int H, int W,
                                     float* __restrict__ dst, int d, int h, int w) {
  const long long total = (long long)C * d * h * w;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int ox = (int)(e % w);
    long long q = e / w;
    const int oy = (int)(q % h);
    q /= h;
    const int oz = (int)(q % d);
    const int c = (int)(q / d);
    const AxisMap mz = axis_map(oz, D, d), my = axis_map(oy, H, h), mx = axis_map(ox, W, w);
    const float* s = src + (long long)c * D * H * W;
    auto at = [&](int z, int y, int x) { return (double)s[((long long)z * H + y) * W + x]; };
    // axis 0 (z) first, then y, then x: the restatement's order
    double vy[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int y = a ? my.i1v : my.i0, x = b ? mx.i1v : mx.i0;
        vy[a][b] = lerp2(at(mz.i0, y, x), at(mz.i1v, y, x), mz.w0, mz.w1);
      }
    const double vx0 = lerp2(vy[0][0], vy[1][0], my.w0, my.w1);
    const double vx1 = lerp2(vy[0][1], vy[1][1], my.w0, my.w1);
    dst[e] = (float)lerp2(vx0, vx1, mx.w0, mx.w1);
  }
}

__device__ __forceinline__ int nearest_idx(int o, int n_in, int n_out) {
  const double z = n_out > 1 ? (double)(n_in - 1) / (double)(n_out - 1) : 0.0;
  int i = (int)floor(__dadd_rn(__dmul_rn((double)o, z), 0.5));
  return i < n_in ? i : n_in - 1;
}

template <typename L>
__global__ void resize_nearest_kernel(const L* __restrict__ src, int D, int H, int W, L* __restrict__ dst, int d,
                                      int h, int w, long long total) {
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int ox = (int)(e % w);
    long long q = e / w;
    const int oy = (int)(q % h);
    q /= h;
    const int oz = (int)(q % d);
    const long long c = q / d;
    dst[e] = src[((c * D + nearest_idx(oz, D, d)) * H + nearest_idx(oy, H, h)) * W + nearest_idx(ox, W, w)];
  }
}

// ----------------------------------------------------------------- phantom
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ double normal_at(uint64_t base, uint64_t i) {
  const uint64_t hsh = splitmix64(i ^ base);
  const double u1 = ((double)(hsh >> 11) + 1.0) * (1.0 / 9007199254740992.0);
  const double u2 = (double)(hsh & 0x1FFFFFull) * (1.0 / 2097152.0);
  return sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
}

constexpr int PH_MAXC = 16, PH_MAXM = 4;
struct PhantomArgs {
  int S, ncls;                       // ncls = number of ellipsoid classes (labels 1..ncls)
  int M;                             // modalities
  double geo[PH_MAXC][6];            // per class: centre z, y, x, radius z, y, x
  float mean[PH_MAXM][PH_MAXC + 1];  // per modality: class mean (index 0 = background)
  float sd[PH_MAXM];
  int absn[PH_MAXM];                 // |N| (PET) instead of N
  uint64_t base[PH_MAXM];            // splitmix64(key) per modality
};

template <typename L>
__global__ void phantom_kernel(PhantomArgs a, L* __restrict__ label, float* __restrict__ image) {
  const long long V = (long long)a.S * a.S * a.S;
  for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < V; v += (long long)gridDim.x * blockDim.x) {
    const int x = (int)(v % a.S), y = (int)((v / a.S) % a.S), z = (int)(v / ((long long)a.S * a.S));
    int lab = 0;
    for (int c = 0; c < a.ncls && lab == 0; ++c) {
      const double dz = ((double)z - a.geo[c][0]) / a.geo[c][3];
      const double dy = ((double)y - a.geo[c][1]) / a.geo[c][4];
      const double dx = ((double)x - a.geo[c][2]) / a.geo[c][5];
      if (__dadd_rn(__dadd_rn(__dmul_rn(dz, dz), __dmul_rn(dy, dy)), __dmul_rn(dx, dx)) <= 1.0) lab = c + 1;
    }
    label[v] = (L)lab;
    for (int m = 0; m < a.M; ++m) {
      double n = normal_at(a.base[m], (uint64_t)v);
      if (a.absn[m]) n = fabs(n);
      image[(long long)m * V + v] = (float)((double)a.mean[m][lab] + (double)a.sd[m] * n);
    }
  }
}

int grid_of(long long total) {
  long long b = (total + 255) / 256;
  return (int)(b < 8192 ? (b < 1 ? 1 : b) : 8192);
}

uint64_t splitmix64_host(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

}  // namespace

extern "C" {

long long mmseg_normalize_ws_bytes(void) { return (long long)(NB + 2) * (long long)sizeof(double); }

int mmseg_modality_normalize(float* x, long long V, int kind, double lo, double hi, void* ws, void* stream) {
  MMSEG_REQUIRE(V >= 1, "modality_normalize: empty volume");
  hipStream_t s = (hipStream_t)stream;
  if (kind == 0) {
    MMSEG_REQUIRE(hi > lo, "modality_normalize: CT window width must be > 0");
    MMSEG_LAUNCH(ct_window_kernel, dim3(grid_of(V)), dim3(256), 0, s, x, V, (float)lo, (float)hi,
                       (float)(hi - lo));
    return mmseg::check_launch("ct_window");
  }
  MMSEG_REQUIRE(kind == 1 || kind == 2, "modality_normalize: kind 0 (CT), 1 (PET), 2 (z-score)");
  MMSEG_REQUIRE(ws != nullptr, "modality_normalize: workspace (mmseg_normalize_ws_bytes())");
  double* part = (double*)ws;
  double* stats = part + NB;
  if (kind == 1) {
    MMSEG_LAUNCH(stat_partial_kernel, dim3(NB), dim3(256), 0, s, x, V, 0, stats, part);
    MMSEG_LAUNCH(stat_final_kernel, dim3(1), dim3(64), 0, s, part, NB, 0, V, stats);
    MMSEG_LAUNCH(scale_kernel, dim3(grid_of(V)), dim3(256), 0, s, x, V, 0, stats);
  } else {
    MMSEG_LAUNCH(stat_partial_kernel, dim3(NB), dim3(256), 0, s, x, V, 1, stats, part);
    MMSEG_LAUNCH(stat_final_kernel, dim3(1), dim3(64), 0, s, part, NB, 1, V, stats);
    MMSEG_LAUNCH(stat_partial_kernel, dim3(NB), dim3(256), 0, s, x, V, 2, stats, part);
    MMSEG_LAUNCH(stat_final_kernel, dim3(1), dim3(64), 0, s, part, NB, 2, V, stats);
    MMSEG_LAUNCH(scale_kernel, dim3(grid_of(V)), dim3(256), 0, s, x, V, 1, stats);
  }
  return mmseg::check_launch("modality_normalize");
}

int mmseg_resize_linear(const float* src, int C, int D, int H, int W, float* dst, int d, int h, int w, void* stream) {
  MMSEG_REQUIRE(C >= 1 && D >= 1 && H >= 1 && W >= 1 && d >= 1 && h >= 1 && w >= 1, "resize_linear: empty shape");
  const long long total = (long long)C * d * h * w;
  MMSEG_LAUNCH(resize_linear_kernel, dim3(grid_of(total)), dim3(256), 0, (hipStream_t)stream, src, C, D, H, W,
                     dst, d, h, w);
  return mmseg::check_launch("resize_linear");
}

int mmseg_resize_nearest(const void* src, int label_bytes, int C, int D, int H, int W, void* dst, int d, int h, int w,
                         void* stream) {
  MMSEG_REQUIRE(label_bytes == 8 || label_bytes == 1, "resize_nearest: int64 or uint8 labels");
  const long long total = (long long)C * d * h * w;
  hipStream_t s = (hipStream_t)stream;
  if (label_bytes == 8)
    MMSEG_LAUNCH(resize_nearest_kernel<int64_t>, dim3(grid_of(total)), dim3(256), 0, s, (const int64_t*)src, D,
                       H, W, (int64_t*)dst, d, h, w, total);
  else
    MMSEG_LAUNCH(resize_nearest_kernel<uint8_t>, dim3(grid_of(total)), dim3(256), 0, s, (const uint8_t*)src, D,
                       H, W, (uint8_t*)dst, d, h, w, total);
  return mmseg::check_launch("resize_nearest");
}

int mmseg_phantom(int S, int ncls, const double* geo, int M, const float* class_mean, const float* noise_sd,
                  const int* abs_noise, const unsigned long long* keys, void* label, int label_bytes, float* image,
                  void* stream) {
  MMSEG_REQUIRE(S >= 1 && ncls >= 0 && ncls <= PH_MAXC && M >= 1 && M <= PH_MAXM,
                "phantom: 1 <= S, 0 <= classes <= %d, 1 <= modalities <= %d", PH_MAXC, PH_MAXM);
  MMSEG_REQUIRE(label_bytes == 8 || label_bytes == 1, "phantom: int64 or uint8 labels");
  PhantomArgs a{};
  a.S = S;
  a.ncls = ncls;
  a.M = M;
  for (int c = 0; c < ncls; ++c)
    for (int k = 0; k < 6; ++k) a.geo[c][k] = geo[c * 6 + k];
  for (int m = 0; m < M; ++m) {
    for (int c = 0; c <= ncls; ++c) a.mean[m][c] = class_mean[m * (ncls + 1) + c];
    a.sd[m] = noise_sd[m];
    a.absn[m] = abs_noise[m];
    a.base[m] = splitmix64_host((uint64_t)keys[m]);
  }
  const long long V = (long long)S * S * S;
  hipStream_t s = (hipStream_t)stream;
  if (label_bytes == 8)
    MMSEG_LAUNCH(phantom_kernel<int64_t>, dim3(grid_of(V)), dim3(256), 0, s, a, (int64_t*)label, image);
  else
    MMSEG_LAUNCH(phantom_kernel<uint8_t>, dim3(grid_of(V)), dim3(256), 0, s, a, (uint8_t*)label, image);
  return mmseg::check_launch("phantom");
}

}  // extern "C"
