// HBM-bound kernels of the ConvBlock3D / DownBlock3D / DualEncoder fusion path.
//
//   InstanceNorm3d(affine=False, eps=1e-5, biased variance) + ReLU
//       (reference unet.py:34-35,45,53-60)       -> instnorm_stats / _relu_fwd
//   its backward (+ ReLU mask)                    -> instnorm_relu_bwd_{reduce,apply}
//       with the MaxPool3d(2) backward (unet.py:73) and the fusion backward
//       (dual_encoder.py:193-195 mean / 184-186 add / 188-191 attention) fused
//       into the dy gather, so neither the pooled gradient nor the fused-level
//       gradient is ever materialised per modality.
//   MaxPool3d(2) forward with argmax (ties -> first in z,y,x scan order)
//   modality fusion forward: weighted sum over M level tensors
//   CrossModalAttention gate (dual_encoder.py:207-254): pooled mean -> Linear ->
//       ReLU -> Linear -> softmax, and its backward.
//
// All reductions are two-level and fixed-order (per-block partials, then a
// single-thread-per-output sweep), so results are bitwise reproducible.
#include "mmseg_common.h"

#include <algorithm>

#include <stdlib.h>
#include <type_traits>

namespace {

// ------------------------------------------------------------------ stats
// Welford / Chan statistics: each thread keeps (n, mean, M2) for its 8
// channels; lanes are merged in a fixed order inside the block and chunks in a
// fixed order in the finalize (double).  A shifted-sums formulation is NOT
// used: convolution outputs are far from stationary near the volume border, so
// any single shift value can sit many sigmas from the channel mean and the
// E[x^2]-E[x]^2 cancellation then costs the gradients ~1e-2 accuracy.
// Block = (256 / C8) voxel lanes x C8 channel groups; a thread owns 8 channels
// of one sample and walks voxels v0+vl, v0+vl+lanes_v, ... of its chunk,
// issuing UNR independent 16-B loads before consuming them (the HBM latency is
// hidden by loads in flight, not by occupancy alone).
constexpr int UNR = 4;

template <typename T>
__global__ void in_stats_partial(const T* __restrict__ x, int ld, int V, int C, int vpc, float* __restrict__ part) {
  const int n = blockIdx.y, chunk = blockIdx.x, nchunk = gridDim.x;
  const int C8 = C >> 3;
  const int lanes_v = 256 / C8;
  const int tid = threadIdx.x;
  const int cg = tid % C8, vl = tid / C8;
  const T* xn = x + (long long)n * V * ld + cg * 8;
  float mu[8], m2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mu[j] = 0.f;
    m2[j] = 0.f;
  }
  float cnt = 0.f;
  const int v0 = chunk * vpc;
  const int v1 = v0 + vpc < V ? v0 + vpc : V;
  auto upd = [&](const V8<T>& a) {
    cnt += 1.f;
    const float inv = 1.f / cnt;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float xv = a.get(j);
      const float d = xv - mu[j];
      mu[j] = fmaf(d, inv, mu[j]);
      m2[j] = fmaf(d, xv - mu[j], m2[j]);
    }
  };
  if (vl < lanes_v) {
    int v = v0 + vl;
    for (; v + (UNR - 1) * lanes_v < v1; v += UNR * lanes_v) {
      V8<T> a[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) a[u].load(xn + (long long)(v + u * lanes_v) * ld);
#pragma unroll
      for (int u = 0; u < UNR; ++u) upd(a[u]);
    }
    for (; v < v1; v += lanes_v) {
      V8<T> a;
      a.load(xn + (long long)v * ld);
      upd(a);
    }
  }
  __shared__ float red[2][256 * 8];
  __shared__ float rcnt[256];
  if ((C8 & (C8 - 1)) == 0 && C8 <= 32) {
    // power-of-two channel groups: the voxel lanes of a wave are merged by a
    // shuffle tree (lane l absorbs lane l+o, o = 32 .. C8: lower voxel lanes
    // stay first, fixed order), then lanes < C8 of the 4 waves go through LDS
    // and one thread per channel merges the 4 waves in order.  The serial
    // 64-lane merge below cost ~2 us per block at C = 32.
    for (int o = 32; o >= C8; o >>= 1) {
      const float nb = __shfl_down(cnt, o, 64);
      const float nn = cnt + nb;
      const float fb = nn > 0.f ? nb / nn : 0.f;
      const float fab = nn > 0.f ? cnt * fb : 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float mb = __shfl_down(mu[j], o, 64), sb = __shfl_down(m2[j], o, 64);
        const float delta = mb - mu[j];
        mu[j] = fmaf(delta, fb, mu[j]);
        m2[j] = m2[j] + sb + delta * delta * fab;
      }
      cnt = nn;
    }
    const int lane = tid & 63, wave = tid >> 6;
    if (lane < C8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        red[0][(wave * C8 + lane) * 8 + j] = mu[j];
        red[1][(wave * C8 + lane) * 8 + j] = m2[j];
      }
      rcnt[wave * C8 + lane] = cnt;
    }
    __syncthreads();
    if (tid < C) {
      const int g = tid >> 3, j = tid & 7;
      float na = 0.f, ma = 0.f, sa = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const int t = w * C8 + g;
        const float nb = rcnt[t];
        if (nb == 0.f) continue;
        const float mb = red[0][t * 8 + j], sb = red[1][t * 8 + j];
        const float nn = na + nb;
        const float delta = mb - ma;
        ma = ma + delta * (nb / nn);
        sa = sa + sb + delta * delta * (na * nb / nn);
        na = nn;
      }
      float* p = part + (((long long)n * nchunk + chunk) * C + tid) * 2;
      p[0] = ma;
      p[1] = sa;
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][tid * 8 + j] = mu[j];
    red[1][tid * 8 + j] = m2[j];
  }
  rcnt[tid] = (vl < lanes_v) ? cnt : 0.f;
  __syncthreads();
  // one thread per channel merges the voxel lanes in fixed order (Chan)
  for (int c = tid; c < C; c += 256) {
    const int g = c >> 3, j = c & 7;
    float na = 0.f, ma = 0.f, sa = 0.f;
    for (int l = 0; l < lanes_v; ++l) {
      const int t = l * C8 + g;
      const float nb = rcnt[t];
      if (nb == 0.f) continue;
      const float mb = red[0][t * 8 + j], sb = red[1][t * 8 + j];
      const float nn = na + nb;
      const float delta = mb - ma;
      ma = ma + delta * (nb / nn);
      sa = sa + sb + delta * delta * (na * nb / nn);
      na = nn;
    }
    float* p = part + (((long long)n * nchunk + chunk) * C + c) * 2;
    p[0] = ma;
    p[1] = sa;
  }
}

__device__ __forceinline__ void load8f(const float* p, float* d) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w;
  d[4] = b.x; d[5] = b.y; d[6] = b.z; d[7] = b.w;
}

// one 256-thread block per (n, c): fixed-order Chan merge of the chunk partials in double
// (each thread its chunks in order, a fixed butterfly per wave, then the 4 waves in order;
// one wave per (n, c) walked ~14 dependent chunk loads per lane at 96^3)
template <typename T>
__global__ void in_stats_finalize(const T* __restrict__ x, int ld, long long V, int N, int C, int nchunk,
                                  long long vpc, const float* __restrict__ part, float eps, float* __restrict__ mean,
                                  int mean_ld, float* __restrict__ rstd) {
  const int idx = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = idx / C, c = idx - n * C;
  double na = 0.0, ma = 0.0, sa = 0.0;
  for (int k = threadIdx.x; k < nchunk; k += 256) {   // each thread: its chunks in order
    const float* p = part + (((long long)n * nchunk + k) * C + c) * 2;
    const long long v0 = (long long)k * vpc;
    const long long v1 = v0 + vpc < V ? v0 + vpc : V;
    const double nb = (double)(v1 - v0);
    if (nb <= 0) continue;
    const double nn = na + nb, delta = (double)p[0] - ma;
    ma += delta * (nb / nn);
    sa += (double)p[1] + delta * delta * (na * nb / nn);
    na = nn;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {          // fixed butterfly: deterministic Chan merge across lanes
    const double nb = __shfl_xor(na, o, 64), mb = __shfl_xor(ma, o, 64), sb = __shfl_xor(sa, o, 64);
    const double nn = na + nb;
    if (nn > 0) {
      // order the pair by lane id so both partners compute the bitwise-same result
      const bool lo = (lane & o) == 0;
      const double n1 = lo ? na : nb, m1 = lo ? ma : mb, s1 = lo ? sa : sb;
      const double n2 = lo ? nb : na, m2 = lo ? mb : ma, s2 = lo ? sb : sa;
      const double delta = m2 - m1;
      ma = m1 + delta * (n2 / nn);
      sa = s1 + s2 + delta * delta * (n1 * n2 / nn);
      na = nn;
    }
  }
  __shared__ double wred[4][3];
  if (lane == 0) {
    wred[wave][0] = na;
    wred[wave][1] = ma;
    wred[wave][2] = sa;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  na = 0.0; ma = 0.0; sa = 0.0;
  for (int w = 0; w < 4; ++w) {
    const double nb = wred[w][0];
    if (nb <= 0) continue;
    const double nn = na + nb, delta = wred[w][1] - ma;
    ma += delta * (nb / nn);
    sa += wred[w][2] + delta * delta * (na * nb / nn);
    na = nn;
  }
  const double var = sa / (double)V;
  mean[(long long)n * mean_ld + c] = (float)ma;
  if (rstd) rstd[idx] = (float)(1.0 / sqrt(var + (double)eps));
}

// Statistics from equal-count per-brick partials (mean_b, M2_b) written by the
// brick conv epilogue: one wave per (n, c); mean = avg(mean_b), M2 = sum M2_b +
// cnt * sum (mean_b - mean)^2 (Chan for equal counts), fp64, fixed lane order.
__global__ void in_stats_from_bricks(const float* __restrict__ part, int N, int C, int nb, int cnt, float eps,
                                     float* __restrict__ mean, int mean_ld, float* __restrict__ rstd) {
  const int idx = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (idx >= N * C) return;
  const int n = idx / C, c = idx - n * C;
  const float* p = part + ((long long)n * nb * C + c) * 2;
  double sm = 0.0;
  for (int b = lane; b < nb; b += 64) sm += (double)p[(long long)b * C * 2];
  sm = wave_sum_d(sm);
  const double mu = sm / (double)nb;
  double m2 = 0.0;
  for (int b = lane; b < nb; b += 64) {
    const double d = (double)p[(long long)b * C * 2] - mu;
    m2 += (double)p[(long long)b * C * 2 + 1] + (double)cnt * d * d;
  }
  m2 = wave_sum_d(m2);
  if (lane != 0) return;
  mean[(long long)n * mean_ld + c] = (float)mu;
  if (rstd) rstd[idx] = (float)(1.0 / sqrt(m2 / ((double)nb * cnt) + (double)eps));
}

// y = relu((x - mean) * rstd); a thread owns 8 channels of one sample (their
// mean / rstd stay in registers) and UNR voxels per step; grid (chunks, N).
template <typename T, bool RELU = true>
__global__ void in_relu_apply(const T* __restrict__ x, int ldx, T* __restrict__ y, int ldy, int V, int C, int vpc,
                              const float* __restrict__ mean, const float* __restrict__ rstd) {
  const int n = blockIdx.y;
  const int C8 = C >> 3, lanes_v = 256 / C8;
  const int cg = threadIdx.x % C8, vl = threadIdx.x / C8;
  if (vl >= lanes_v) return;
  float mu[8], rs[8];
  load8f(mean + n * C + cg * 8, mu);
  load8f(rstd + n * C + cg * 8, rs);
  const T* xn = x + (long long)n * V * ldx + cg * 8;
  T* yn = y + (long long)n * V * ldy + cg * 8;
  const int v0 = blockIdx.x * vpc;
  const int v1 = v0 + vpc < V ? v0 + vpc : V;
  for (int vb = v0 + vl; vb < v1; vb += UNR * lanes_v) {
    V8<T> a[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u)
      if (vb + u * lanes_v < v1) a[u].load(xn + (long long)(vb + u * lanes_v) * ldx);
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      if (vb + u * lanes_v >= v1) break;
      V8<T> o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float h = (a[u].get(j) - mu[j]) * rs[j];
        o.set(j, (!RELU || h > 0.f) ? h : 0.f);
      }
      o.store(yn + (long long)(vb + u * lanes_v) * ldy);
    }
  }
}

// --------------------------------------------------------------- maxpool
// 2x2x2, stride 2.  idx = a*4 + b*2 + c (z,y,x), first maximum wins.
// NORM: x is the PRE-norm activation and the pooled values are relu((x - mean) * rstd) rounded to T, i.e.
// exactly in_relu_apply's output, so values and argmax (ties included) equal pooling the materialised
// InstanceNorm + ReLU output, which then never has to be written (DualEncoder mean / add fusion).
template <typename T, bool NORM = false>
__global__ void maxpool2_fwd(const T* __restrict__ x, int ldx, T* __restrict__ y, int ldy,
                             uint8_t* __restrict__ idx, int N, int D, int H, int W, int C,
                             const float* __restrict__ mean = nullptr, const float* __restrict__ rstd = nullptr) {
  const int C8 = C >> 3;
  const int Do = D >> 1, Ho = H >> 1, Wo = W >> 1;
  // 32-bit item index (the host requires N * Vo * C8 < 2^31): the former 64-bit divisions were most of the
  // kernel's VALU work
  const int total = N * Do * Ho * Wo * C8;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int cg = i % C8;
    int q = i / C8;
    const int xo = q % Wo;
    q /= Wo;
    const int yo = q % Ho;
    q /= Ho;
    const int zo = q % Do;
    const int n = q / Do;
    const long long in0 = ((long long)(n * D + 2 * zo) * H + 2 * yo) * (long long)W + 2 * xo;
    float best[8];
    uint8_t bi[8];
    float mu[8], rs[8];
    if constexpr (NORM) {
      load8f(mean + n * C + cg * 8, mu);
      load8f(rstd + n * C + cg * 8, rs);
    }
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const long long vin = in0 + ((long long)(t >> 2) * H + ((t >> 1) & 1)) * W + (t & 1);
      V8<T> a;
      a.load(x + vin * ldx + cg * 8);
      if constexpr (NORM) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float h = (a.get(j) - mu[j]) * rs[j];
          a.set(j, h > 0.f ? h : 0.f);
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        // torch CPU max_pool3d: (val > maxval) || isnan(val) replaces
        const float v = a.get(j);
        if (t == 0 || v > best[j] || v != v) {
          best[j] = v;
          bi[j] = (uint8_t)t;
        }
      }
    }
    V8<T> o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o.set(j, best[j]);
    const long long vo = ((long long)(n * Do + zo) * Ho + yo) * Wo + xo;
    o.store(y + vo * ldy + cg * 8);
    uint2 packed;
    packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
    packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
    *reinterpret_cast<uint2*>(idx + vo * C + cg * 8) = packed;
  }
}

// ------------------------------------------------------------- dy gather
// dy(n, v, c) = scale1 * alpha1[n] * p1[n,v,c] + beta[n,c]
//             + (pool_idx[n, pool(v), c] == sub(v) ? pool_dy[n, pool(v), c] : 0)
struct DySrc {
  const void* p1;
  int ld1;
  float scale1;
  const float* alpha1;   // [N] (stride alpha_stride) or null
  int alpha_stride;
  const float* beta;     // [N][C] (stride beta_stride per n) or null
  int beta_stride;
  const void* pool_dy;   // [N][Vo][C] with ld pool_ld, or null
  int pool_ld;
  const uint8_t* pool_idx;  // [N][Vo][C]
  int p1_nmod;           // > 0: p1 holds p1_nmod samples, sample n reads p1 sample n % p1_nmod (the fused level's
                         // gradient shared by the M modality groups of a grouped backward)
  float slope;           // ACT 2: the LeakyReLU's negative slope
  // > 1 (with p1_nmod): the partial / apply grids are (chunks x gsplit, p1_nmod) -- the gsplit modality samples
  // that read one p1 sample take adjacent blocks of each chunk, so the second read of that p1 chunk is served by
  // the Infinity Cache instead of HBM (launched sample-major, the re-read came ~2 samples = 240 MB later)
  int gsplit;
};

// (sample, chunk, chunks) of a partial / apply block (DySrc::gsplit)
__device__ __forceinline__ void in_block(const DySrc& s, int& n, int& chunk, int& nchunk) {
  if (s.gsplit > 1) {
    chunk = (int)blockIdx.x / s.gsplit;
    n = ((int)blockIdx.x % s.gsplit) * s.p1_nmod + (int)blockIdx.y;
    nchunk = (int)gridDim.x / s.gsplit;
  } else {
    n = (int)blockIdx.y;
    chunk = (int)blockIdx.x;
    nchunk = (int)gridDim.x;
  }
}

// gradient through the activation that follows the norm (h: the normalised value; an activation keeps the sign,
// so h > 0 is where its output is > 0): ACT 0 none, 1 ReLU, 2 LeakyReLU
template <int ACT>
__device__ __forceinline__ float act_grad(float h, float dy, float slope) {
  if constexpr (ACT == 0) return dy;
  else if constexpr (ACT == 1) return h > 0.f ? dy : 0.f;
  else return h > 0.f ? dy : dy * slope;
}

// 8 zeros into a row's channel padding (whole-row writes; see mmseg_instnorm_act_bwd)
template <typename T>
__device__ __forceinline__ void store_zero8(T* p) {
  V8<T> z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z.set(j, 0.f);
  z.store(p);
}

// Per-thread view of a DySrc for one sample and one 8-channel group: the
// scale, beta and base pointers are resolved once, the per-voxel work is the
// loads and the pool-window test.
template <typename T>
struct DyCtx {
  const T* p1;
  int ld1;
  float sc;
  float beta[8];
  bool has_beta;
  const T* pdy;
  int pool_ld;
  const uint8_t* pidx;
  int C, H, W, Ho, Wo, HWo;

  __device__ __forceinline__ DyCtx(const DySrc& s, int n, int V, int cg, int C_, int D, int H_, int W_) {
    C = C_;
    H = H_;
    W = W_;
    const int n1 = s.p1_nmod > 0 ? n % s.p1_nmod : n;
    p1 = s.p1 ? reinterpret_cast<const T*>(s.p1) + (long long)n1 * V * s.ld1 + cg * 8 : nullptr;
    ld1 = s.ld1;
    sc = s.scale1 * (s.alpha1 ? s.alpha1[n * s.alpha_stride] : 1.f);
    has_beta = s.beta != nullptr;
#pragma unroll
    for (int j = 0; j < 8; ++j) beta[j] = has_beta ? s.beta[n * s.beta_stride + cg * 8 + j] : 0.f;
    Ho = H >> 1;
    Wo = W >> 1;
    HWo = Ho * Wo;
    const long long Vo = (long long)(D >> 1) * HWo;
    pdy = s.pool_dy ? reinterpret_cast<const T*>(s.pool_dy) + (long long)n * Vo * s.pool_ld + cg * 8 : nullptr;
    pool_ld = s.pool_ld;
    pidx = s.pool_dy ? s.pool_idx + (long long)n * Vo * C + cg * 8 : nullptr;
  }

  // raw loads for voxel v (issued early), then combine
  struct Raw {
    V8<T> a, pd;
    uint2 id;
    uint8_t sub;
  };
  __device__ __forceinline__ void load(int v, Raw& r) const {
    if (p1) r.a.load(p1 + (long long)v * ld1);
    if (pdy) {
      const int x = v % W;
      const int q = v / W;
      const int y = q % H, z = q / H;
      const int vo = (z >> 1) * HWo + (y >> 1) * Wo + (x >> 1);
      r.sub = (uint8_t)(((z & 1) << 2) | ((y & 1) << 1) | (x & 1));
      r.pd.load(pdy + (long long)vo * pool_ld);
      r.id = *reinterpret_cast<const uint2*>(pidx + (long long)vo * C);
    }
  }
  __device__ __forceinline__ void combine(const Raw& r, float* dy) const {
#pragma unroll
    for (int j = 0; j < 8; ++j) dy[j] = (p1 ? r.a.get(j) * sc : 0.f) + beta[j];
    if (pdy) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t w = j < 4 ? r.id.x : r.id.y;
        const uint8_t id = (uint8_t)((w >> ((j & 3) * 8)) & 0xff);
        if (id == r.sub) dy[j] += r.pd.get(j);
      }
    }
  }
};

// partial sums of g and g*xhat, g = dy * [xhat > 0]
template <typename T, int ACT = 1>
__global__ void in_bwd_partial(const T* __restrict__ x, int ldx, const float* __restrict__ mean,
                               const float* __restrict__ rstd, DySrc s, int V, int C, int D, int H, int W, int vpc,
                               float* __restrict__ part) {
  int n, chunk, nchunk;
  in_block(s, n, chunk, nchunk);
  const int C8 = C >> 3;
  const int lanes_v = 256 / C8;
  const int tid = threadIdx.x;
  const int cg = tid % C8, vl = tid / C8;
  float sg[8], sgx[8], mu[8], rs[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sg[j] = 0.f;
    sgx[j] = 0.f;
  }
  load8f(mean + n * C + cg * 8, mu);
  load8f(rstd + n * C + cg * 8, rs);
  const DyCtx<T> dc(s, n, V, cg, C, D, H, W);
  const T* xn = x + (long long)n * V * ldx + cg * 8;
  const int v0 = chunk * vpc;
  const int v1 = v0 + vpc < V ? v0 + vpc : V;
  if (vl < lanes_v) {
    for (int vb = v0 + vl; vb < v1; vb += UNR * lanes_v) {
      V8<T> a[UNR];
      typename DyCtx<T>::Raw r[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u)
        if (vb + u * lanes_v < v1) {
          a[u].load(xn + (long long)(vb + u * lanes_v) * ldx);
          dc.load(vb + u * lanes_v, r[u]);
        }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        if (vb + u * lanes_v >= v1) break;
        float dy[8];
        dc.combine(r[u], dy);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float h = (a[u].get(j) - mu[j]) * rs[j];
          const float g = act_grad<ACT>(h, dy[j], s.slope);
          sg[j] += g;
          sgx[j] = fmaf(g, h, sgx[j]);
        }
      }
    }
  }
  __shared__ float red[2][256 * 8];
  if ((C8 & (C8 - 1)) == 0 && C8 <= 32) {
    // shuffle tree over the voxel lanes of each wave (fixed order), then the 4 waves in order
    for (int o = 32; o >= C8; o >>= 1) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sg[j] += __shfl_down(sg[j], o, 64);
        sgx[j] += __shfl_down(sgx[j], o, 64);
      }
    }
    const int lane = tid & 63, wave = tid >> 6;
    if (lane < C8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        red[0][(wave * C8 + lane) * 8 + j] = sg[j];
        red[1][(wave * C8 + lane) * 8 + j] = sgx[j];
      }
    }
    __syncthreads();
    if (tid < C) {
      const int g = tid >> 3, j = tid & 7;
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        a += red[0][(w * C8 + g) * 8 + j];
        b += red[1][(w * C8 + g) * 8 + j];
      }
      float* p = part + (((long long)n * nchunk + chunk) * C + tid) * 2;
      p[0] = a;
      p[1] = b;
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][tid * 8 + j] = sg[j];
    red[1][tid * 8 + j] = sgx[j];
  }
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    const int g = c >> 3, j = c & 7;
    float a = 0.f, b = 0.f;
    for (int l = 0; l < lanes_v; ++l) {
      a += red[0][(l * C8 + g) * 8 + j];
      b += red[1][(l * C8 + g) * 8 + j];
    }
    float* p = part + (((long long)n * nchunk + chunk) * C + c) * 2;
    p[0] = a;
    p[1] = b;
  }
}

// one 256-thread block per (n, c): fixed-order double sums of the chunk partials
__global__ void in_bwd_finalize(const float* __restrict__ part, int N, int C, int nchunk, long long V,
                                float* __restrict__ coef) {
  const int idx = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = idx / C, c = idx - n * C;
  double a = 0.0, b = 0.0;
  for (int k = threadIdx.x; k < nchunk; k += 256) {
    const float* p = part + (((long long)n * nchunk + k) * C + c) * 2;
    a += p[0];
    b += p[1];
  }
  a = wave_sum_d(a);
  b = wave_sum_d(b);
  __shared__ double wred[4][2];
  if (lane == 0) {
    wred[wave][0] = a;
    wred[wave][1] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    a = (wred[0][0] + wred[1][0]) + (wred[2][0] + wred[3][0]);
    b = (wred[0][1] + wred[1][1]) + (wred[2][1] + wred[3][1]);
    coef[idx * 2 + 0] = (float)(a / (double)V);
    coef[idx * 2 + 1] = (float)(b / (double)V);
  }
}

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)); same thread layout as the apply kernels
template <typename T, int ACT = 1, bool ZP = false>
__global__ void in_bwd_apply(const T* __restrict__ x, int ldx, const float* __restrict__ mean,
                             const float* __restrict__ rstd, DySrc s, const float* __restrict__ coef, T* __restrict__ dx,
                             int lddx, int V, int C, int D, int H, int W, int vpc, int npad) {
  int n, chunk, nchunk;
  in_block(s, n, chunk, nchunk);
  const int C8 = C >> 3, lanes_v = 256 / C8;
  const int cg = threadIdx.x % C8, vl = threadIdx.x / C8;
  if (vl >= lanes_v) return;
  float mu[8], rs[8], ca[8], cb[8];
  load8f(mean + n * C + cg * 8, mu);
  load8f(rstd + n * C + cg * 8, rs);
  {
    float t[16];
    load8f(coef + (n * C + cg * 8) * 2, t);
    load8f(coef + (n * C + cg * 8) * 2 + 8, t + 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ca[j] = t[2 * j];
      cb[j] = t[2 * j + 1];
    }
  }
  const DyCtx<T> dc(s, n, V, cg, C, D, H, W);
  const T* xn = x + (long long)n * V * ldx + cg * 8;
  T* dxn = dx + (long long)n * V * lddx + cg * 8;
  const int v0 = chunk * vpc;
  const int v1 = v0 + vpc < V ? v0 + vpc : V;
  for (int vb = v0 + vl; vb < v1; vb += UNR * lanes_v) {
    V8<T> a[UNR];
    typename DyCtx<T>::Raw r[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u)
      if (vb + u * lanes_v < v1) {
        a[u].load(xn + (long long)(vb + u * lanes_v) * ldx);
        dc.load(vb + u * lanes_v, r[u]);
      }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      if (vb + u * lanes_v >= v1) break;
      float dy[8];
      dc.combine(r[u], dy);
      V8<T> o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float h = (a[u].get(j) - mu[j]) * rs[j];
        const float g = act_grad<ACT>(h, dy[j], s.slope);
        o.set(j, rs[j] * (g - ca[j] - h * cb[j]));
      }
      o.store(dxn + (long long)(vb + u * lanes_v) * lddx);
      if constexpr (ZP) {   // whole-row writes (a separate instantiation: the plain one keeps its code)
        if (cg < npad) store_zero8(dxn + (long long)(vb + u * lanes_v) * lddx + C);   // (dxn is at channel 8 cg)
      }
    }
  }
}

// The UnetResBlock tail's backward, first pass (y = lrelu(IN(xa) + IN(xb) | + residual)): g = dy * (y > 0 ? 1 :
// slope), stored (the norms' apply passes and the residual branch read it), and in the same pass the partial sums
// (sum g, sum g xhat) of the InstanceNorm backward of xa and, NX = 2, of xb -- over g as stored, with
// in_bwd_partial's chunks, per-thread voxel order and reduction tree, so the partials and everything after them
// are those of lrelu_bwd_kernel + in_bwd_partial bit for bit, without the separate passes over g.
template <typename T, int NX, bool ZP>
__global__ __launch_bounds__(256) void lrelu_bwd_in_partial(const T* __restrict__ y, int ldy,
                                                            const T* __restrict__ dy, int lddy, T* __restrict__ g,
                                                            int ldg, float slope, const T* __restrict__ xa, int lda,
                                                            const float* __restrict__ ma, const float* __restrict__ ra,
                                                            float* __restrict__ pa, const T* __restrict__ xb, int ldb,
                                                            const float* __restrict__ mb, const float* __restrict__ rb,
                                                            float* __restrict__ pb, int V, int C, int vpc,
                                                            int npad) {
  constexpr int K = 1 + NX;    // sum g, sum g xhat_a (, sum g xhat_b)
  const int n = blockIdx.y, chunk = blockIdx.x, nchunk = gridDim.x;
  const int C8 = C >> 3, lanes_v = 256 / C8;
  const int tid = threadIdx.x, cg = tid % C8, vl = tid / C8;
  float acc[K][8], mua[8], rsa[8], mub[8], rsb[8];
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[k][j] = 0.f;
  load8f(ma + n * C + cg * 8, mua);
  load8f(ra + n * C + cg * 8, rsa);
  if constexpr (NX > 1) {
    load8f(mb + n * C + cg * 8, mub);
    load8f(rb + n * C + cg * 8, rsb);
  }
  const long long row0 = (long long)n * V;
  const int v0 = chunk * vpc;
  const int v1 = v0 + vpc < V ? v0 + vpc : V;
  if (vl < lanes_v) {
    for (int vb = v0 + vl; vb < v1; vb += UNR * lanes_v) {
      V8<T> vy[UNR], vd[UNR], va[UNR], vx[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u)
        if (vb + u * lanes_v < v1) {
          const long long t = row0 + vb + u * lanes_v;
          vy[u].load(y + t * ldy + cg * 8);
          vd[u].load(dy + t * lddy + cg * 8);
          va[u].load(xa + t * lda + cg * 8);
          if constexpr (NX > 1) vx[u].load(xb + t * ldb + cg * 8);
        }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        if (vb + u * lanes_v >= v1) break;
        const long long t = row0 + vb + u * lanes_v;
        V8<T> gv;
#pragma unroll
        for (int j = 0; j < 8; ++j) gv.set(j, vy[u].get(j) > 0.f ? vd[u].get(j) : vd[u].get(j) * slope);
        gv.store(g + t * ldg + cg * 8);
        if constexpr (ZP) {
          if (cg < npad) store_zero8(g + t * ldg + C + cg * 8);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float gg = gv.get(j);
          const float h = (va[u].get(j) - mua[j]) * rsa[j];
          acc[0][j] += gg;
          acc[1][j] = fmaf(gg, h, acc[1][j]);
          if constexpr (NX > 1) {
            const float h2 = (vx[u].get(j) - mub[j]) * rsb[j];
            acc[2][j] = fmaf(gg, h2, acc[2][j]);
          }
        }
      }
    }
  }
  // in_bwd_partial's reduction, K sums at once
  __shared__ float red[K][256 * 8];
  float* const pout[2] = {pa + ((long long)n * nchunk + chunk) * C * 2,
                          NX > 1 ? pb + ((long long)n * nchunk + chunk) * C * 2 : nullptr};
  if ((C8 & (C8 - 1)) == 0 && C8 <= 32) {
    for (int o = 32; o >= C8; o >>= 1) {
#pragma unroll
      for (int k = 0; k < K; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[k][j] += __shfl_down(acc[k][j], o, 64);
    }
    const int lane = tid & 63, wave = tid >> 6;
    if (lane < C8) {
#pragma unroll
      for (int k = 0; k < K; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j) red[k][(wave * C8 + lane) * 8 + j] = acc[k][j];
    }
    __syncthreads();
    if (tid < C) {
      const int gi = tid >> 3, j = tid & 7;
      float s[K];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        s[k] = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) s[k] += red[k][(w * C8 + gi) * 8 + j];
      }
#pragma unroll
      for (int x = 0; x < NX; ++x) {
        pout[x][tid * 2] = s[0];
        pout[x][tid * 2 + 1] = s[1 + x];
      }
    }
    return;
  }
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) red[k][tid * 8 + j] = acc[k][j];
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    const int gi = c >> 3, j = c & 7;
    float s[K];
#pragma unroll
    for (int k = 0; k < K; ++k) s[k] = 0.f;
    for (int l = 0; l < lanes_v; ++l)
#pragma unroll
      for (int k = 0; k < K; ++k) s[k] += red[k][(l * C8 + gi) * 8 + j];
#pragma unroll
    for (int x = 0; x < NX; ++x) {
      pout[x][c * 2] = s[0];
      pout[x][c * 2 + 1] = s[1 + x];
    }
  }
}

// ------------------------------------------------- small-volume fused IN
// The 12^3 / 6^3 levels (V <= 4096 voxels per sample): one 256-thread block per (8-channel group, sample)
// holds the whole reduction, so InstanceNorm forward is ONE launch (statistics, then the normalised output
// from a second, L2-resident read) instead of partial + finalize + apply, and the backward likewise.
// Per-thread Welford / sums in fp32; lanes merge with a fixed xor-shuffle tree (Chan's formula for the
// Welford pairs), then the 4 waves in order through LDS: deterministic.  (The previous 1024-thread form
// with a 10-level LDS tree and 68 KB of LDS spent most of its time in the tree: ~1.7 voxels per thread.)
constexpr int SMALL_T = 256;

__device__ __forceinline__ void chan_merge(float& cnt, float* mu, float* m2, float nb, const float* mb,
                                           const float* m2b) {
  const float na = cnt, nn = na + nb;
  if (nb > 0.f) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float dl = mb[j] - mu[j];
      mu[j] = mu[j] + dl * (nb / nn);
      m2[j] = m2[j] + m2b[j] + dl * dl * (na * nb / nn);
    }
    cnt = nn;
  }
}

template <typename T, bool RELU>
__global__ __launch_bounds__(SMALL_T) void in_small_fwd(const T* __restrict__ x, int ldx, T* __restrict__ y, int ldy,
                                                       int V, int C, float eps, float* __restrict__ mean,
                                                       int mean_ld, float* __restrict__ rstd) {
  __shared__ float smu[4][8], sm2[4][8], scnt[4], sfin[16];
  const int cg = blockIdx.x, n = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const T* xn = x + (long long)n * V * ldx + cg * 8;
  float mu[8], m2[8], cnt = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) mu[j] = m2[j] = 0.f;
  auto upd = [&](const V8<T>& a) {
    cnt += 1.f;
    const float inv = 1.f / cnt;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float xv = a.get(j), d = xv - mu[j];
      mu[j] = fmaf(d, inv, mu[j]);
      m2[j] = fmaf(d, xv - mu[j], m2[j]);
    }
  };
  int v = tid;
  for (; v + 3 * SMALL_T < V; v += 4 * SMALL_T) {   // 4 loads in flight
    V8<T> a[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u].load(xn + (long long)(v + u * SMALL_T) * ldx);
#pragma unroll
    for (int u = 0; u < 4; ++u) upd(a[u]);
  }
  for (; v < V; v += SMALL_T) {
    V8<T> a;
    a.load(xn + (long long)v * ldx);
    upd(a);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float mb[8], m2b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      mb[j] = __shfl_xor(mu[j], o, 64);
      m2b[j] = __shfl_xor(m2[j], o, 64);
    }
    chan_merge(cnt, mu, m2, __shfl_xor(cnt, o, 64), mb, m2b);
  }
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      smu[wave][j] = mu[j];
      sm2[wave][j] = m2[j];
    }
    scnt[wave] = cnt;
  }
  __syncthreads();
  if (tid < 8) {   // channel tid: the 4 waves in order
    float c0 = scnt[0], m0 = smu[0][tid], q0 = sm2[0][tid];
    for (int w = 1; w < 4; ++w) {
      const float nb = scnt[w], nn = c0 + nb;
      if (nb > 0.f) {
        const float dl = smu[w][tid] - m0;
        m0 = m0 + dl * (nb / nn);
        q0 = q0 + sm2[w][tid] + dl * dl * (c0 * nb / nn);
        c0 = nn;
      }
    }
    const float rs = 1.f / sqrtf(q0 / (float)V + eps);
    sfin[tid] = m0;
    sfin[8 + tid] = rs;
    mean[(long long)n * mean_ld + cg * 8 + tid] = m0;
    rstd[n * C + cg * 8 + tid] = rs;
  }
  __syncthreads();
  float m[8], rs[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    m[j] = sfin[j];
    rs[j] = sfin[8 + j];
  }
  T* yn = y + (long long)n * V * ldy + cg * 8;
  // 4 (L2-resident) loads in flight per thread before the stores: one latency per 4 voxels
  for (int v0 = tid; v0 < V; v0 += 4 * SMALL_T) {
    V8<T> a[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (v0 + u * SMALL_T < V) a[u].load(xn + (long long)(v0 + u * SMALL_T) * ldx);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (v0 + u * SMALL_T >= V) break;
      V8<T> o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float h = (a[u].get(j) - m[j]) * rs[j];
        o.set(j, (!RELU || h > 0.f) ? h : 0.f);
      }
      o.store(yn + (long long)(v0 + u * SMALL_T) * ldy);
    }
  }
}

template <typename T, int ACT>
__global__ __launch_bounds__(SMALL_T) void in_small_bwd(const T* __restrict__ x, int ldx, const float* __restrict__ mean,
                                                       const float* __restrict__ rstd, DySrc s, T* __restrict__ dx,
                                                       int lddx, int V, int C, int D, int H, int W) {
  __shared__ float sa[4][8], sb[4][8], sfin[16];
  const int cg = blockIdx.x, n = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float mu[8], rs[8], ga[8], gb[8];
  load8f(mean + n * C + cg * 8, mu);
  load8f(rstd + n * C + cg * 8, rs);
#pragma unroll
  for (int j = 0; j < 8; ++j) ga[j] = gb[j] = 0.f;
  const DyCtx<T> dc(s, n, V, cg, C, D, H, W);
  const T* xn = x + (long long)n * V * ldx + cg * 8;
  // 4 voxels' loads in flight per thread, consumed in voxel order (the sums' order is unchanged)
  for (int v0 = tid; v0 < V; v0 += 4 * SMALL_T) {
    V8<T> a[4];
    typename DyCtx<T>::Raw r[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (v0 + u * SMALL_T < V) {
        a[u].load(xn + (long long)(v0 + u * SMALL_T) * ldx);
        dc.load(v0 + u * SMALL_T, r[u]);
      }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (v0 + u * SMALL_T >= V) break;
      float dy[8];
      dc.combine(r[u], dy);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float h = (a[u].get(j) - mu[j]) * rs[j];
        const float g = act_grad<ACT>(h, dy[j], s.slope);
        ga[j] += g;
        gb[j] = fmaf(g, h, gb[j]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ga[j] = wave_sum(ga[j]);
    gb[j] = wave_sum(gb[j]);
  }
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sa[wave][j] = ga[j];
      sb[wave][j] = gb[j];
    }
  }
  __syncthreads();
  if (tid < 8) {
    sfin[tid] = (((sa[0][tid] + sa[1][tid]) + sa[2][tid]) + sa[3][tid]) / (float)V;
    sfin[8 + tid] = (((sb[0][tid] + sb[1][tid]) + sb[2][tid]) + sb[3][tid]) / (float)V;
  }
  __syncthreads();
  float ca[8], cb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ca[j] = sfin[j];
    cb[j] = sfin[8 + j];
  }
  T* dxn = dx + (long long)n * V * lddx + cg * 8;
  for (int v0 = tid; v0 < V; v0 += 4 * SMALL_T) {
    V8<T> a[4];
    typename DyCtx<T>::Raw r[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (v0 + u * SMALL_T < V) {
        a[u].load(xn + (long long)(v0 + u * SMALL_T) * ldx);
        dc.load(v0 + u * SMALL_T, r[u]);
      }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (v0 + u * SMALL_T >= V) break;
      float dy[8];
      dc.combine(r[u], dy);
      V8<T> o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float h = (a[u].get(j) - mu[j]) * rs[j];
        const float g = act_grad<ACT>(h, dy[j], s.slope);
        o.set(j, rs[j] * (g - ca[j] - h * cb[j]));
      }
      o.store(dxn + (long long)(v0 + u * SMALL_T) * lddx);
    }
  }
}

// Register-resident forms for V <= VPT * 256 (the 12^3 and 6^3 levels): every voxel of the thread is loaded
// once, up front (one memory latency instead of one per pass and per 4 voxels), kept in registers through the
// statistics and applied from there.  The per-thread accumulation order (voxels tid, tid + 256, ...) and the
// merge trees are those of in_small_fwd / in_small_bwd, so the results are bitwise the same.
template <typename T, bool RELU, int VPT>
__global__ __launch_bounds__(SMALL_T) void in_small_fwd_r(const T* __restrict__ x, int ldx, T* __restrict__ y,
                                                         int ldy, int V, int C, float eps, float* __restrict__ mean,
                                                         int mean_ld, float* __restrict__ rstd) {
  __shared__ float smu[4][8], sm2[4][8], scnt[4], sfin[16];
  const int cg = blockIdx.x, n = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const T* xn = x + (long long)n * V * ldx + cg * 8;
  V8<T> a[VPT];
#pragma unroll
  for (int u = 0; u < VPT; ++u)
    if (tid + u * SMALL_T < V) a[u].load(xn + (long long)(tid + u * SMALL_T) * ldx);
  float mu[8], m2[8], cnt = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) mu[j] = m2[j] = 0.f;
#pragma unroll
  for (int u = 0; u < VPT; ++u) {
    if (tid + u * SMALL_T >= V) break;
    cnt += 1.f;
    const float inv = 1.f / cnt;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float xv = a[u].get(j), d = xv - mu[j];
      mu[j] = fmaf(d, inv, mu[j]);
      m2[j] = fmaf(d, xv - mu[j], m2[j]);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float mb[8], m2b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      mb[j] = __shfl_xor(mu[j], o, 64);
      m2b[j] = __shfl_xor(m2[j], o, 64);
    }
    chan_merge(cnt, mu, m2, __shfl_xor(cnt, o, 64), mb, m2b);
  }
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      smu[wave][j] = mu[j];
      sm2[wave][j] = m2[j];
    }
    scnt[wave] = cnt;
  }
  __syncthreads();
  if (tid < 8) {
    float c0 = scnt[0], m0 = smu[0][tid], q0 = sm2[0][tid];
    for (int w = 1; w < 4; ++w) {
      const float nb = scnt[w], nn = c0 + nb;
      if (nb > 0.f) {
        const float dl = smu[w][tid] - m0;
        m0 = m0 + dl * (nb / nn);
        q0 = q0 + sm2[w][tid] + dl * dl * (c0 * nb / nn);
        c0 = nn;
      }
    }
    const float rs = 1.f / sqrtf(q0 / (float)V + eps);
    sfin[tid] = m0;
    sfin[8 + tid] = rs;
    mean[(long long)n * mean_ld + cg * 8 + tid] = m0;
    rstd[n * C + cg * 8 + tid] = rs;
  }
  __syncthreads();
  float m[8], rs[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    m[j] = sfin[j];
    rs[j] = sfin[8 + j];
  }
  T* yn = y + (long long)n * V * ldy + cg * 8;
#pragma unroll
  for (int u = 0; u < VPT; ++u) {
    if (tid + u * SMALL_T >= V) break;
    V8<T> o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float h = (a[u].get(j) - m[j]) * rs[j];
      o.set(j, (!RELU || h > 0.f) ? h : 0.f);
    }
    o.store(yn + (long long)(tid + u * SMALL_T) * ldy);
  }
}

template <typename T, int ACT, int VPT>
__global__ __launch_bounds__(SMALL_T) void in_small_bwd_r(const T* __restrict__ x, int ldx,
                                                         const float* __restrict__ mean, const float* __restrict__ rstd,
                                                         DySrc s, T* __restrict__ dx, int lddx, int V, int C, int D,
                                                         int H, int W) {
  __shared__ float sa[4][8], sb[4][8], sfin[16];
  const int cg = blockIdx.x, n = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const DyCtx<T> dc(s, n, V, cg, C, D, H, W);
  const T* xn = x + (long long)n * V * ldx + cg * 8;
  V8<T> a[VPT];
  float dy[VPT][8];
  {
    typename DyCtx<T>::Raw r[VPT];
#pragma unroll
    for (int u = 0; u < VPT; ++u)
      if (tid + u * SMALL_T < V) {
        a[u].load(xn + (long long)(tid + u * SMALL_T) * ldx);
        dc.load(tid + u * SMALL_T, r[u]);
      }
#pragma unroll
    for (int u = 0; u < VPT; ++u)
      if (tid + u * SMALL_T < V) dc.combine(r[u], dy[u]);
  }
  float mu[8], rs[8], ga[8], gb[8];
  load8f(mean + n * C + cg * 8, mu);
  load8f(rstd + n * C + cg * 8, rs);
#pragma unroll
  for (int j = 0; j < 8; ++j) ga[j] = gb[j] = 0.f;
#pragma unroll
  for (int u = 0; u < VPT; ++u) {
    if (tid + u * SMALL_T >= V) break;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float h = (a[u].get(j) - mu[j]) * rs[j];
      const float g = act_grad<ACT>(h, dy[u][j], s.slope);
      ga[j] += g;
      gb[j] = fmaf(g, h, gb[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ga[j] = wave_sum(ga[j]);
    gb[j] = wave_sum(gb[j]);
  }
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sa[wave][j] = ga[j];
      sb[wave][j] = gb[j];
    }
  }
  __syncthreads();
  if (tid < 8) {
    sfin[tid] = (((sa[0][tid] + sa[1][tid]) + sa[2][tid]) + sa[3][tid]) / (float)V;
    sfin[8 + tid] = (((sb[0][tid] + sb[1][tid]) + sb[2][tid]) + sb[3][tid]) / (float)V;
  }
  __syncthreads();
  float ca[8], cb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ca[j] = sfin[j];
    cb[j] = sfin[8 + j];
  }
  T* dxn = dx + (long long)n * V * lddx + cg * 8;
#pragma unroll
  for (int u = 0; u < VPT; ++u) {
    if (tid + u * SMALL_T >= V) break;
    V8<T> o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float h = (a[u].get(j) - mu[j]) * rs[j];
      const float g = act_grad<ACT>(h, dy[u][j], s.slope);
      o.set(j, rs[j] * (g - ca[j] - h * cb[j]));
    }
    o.store(dxn + (long long)(tid + u * SMALL_T) * lddx);
  }
}

// ---------------------------------------------------------------- fusion
// out[n,v,c] = sum_m w_m * src_m[n,v,c],  w_m = wconst or wts[n*M + m]
struct FuseSrc {
  const void* p[4];
  int ld[4];
  int M;
  float wconst;
  const float* wts;   // [N][M] or null
  const float* mean[4];   // NORM: per-source InstanceNorm statistics [N][C] (sources are pre-norm, + ReLU)
  const float* rstd[4];
};

template <typename T, bool NORM = false>
__global__ void fuse_fwd(FuseSrc s, T* __restrict__ out, int ldo, long long V, int N, int C) {
  const int C8 = C >> 3;
  const int total = N * (int)V * C8;   // < 2^31 (host check): 32-bit index math
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int cg = i % C8;
    const long long nv = i / C8;
    const int n = (int)(nv / (int)V);
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    for (int m = 0; m < s.M; ++m) {
      V8<T> a;
      a.load(reinterpret_cast<const T*>(s.p[m]) + nv * s.ld[m] + cg * 8);
      if constexpr (NORM) {   // in_relu_apply's value, rounded to T as the materialised output would be
        float mu[8], rs[8];
        load8f(s.mean[m] + n * C + cg * 8, mu);
        load8f(s.rstd[m] + n * C + cg * 8, rs);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float h = (a.get(j) - mu[j]) * rs[j];
          a.set(j, h > 0.f ? h : 0.f);
        }
      }
      const float w = s.wts ? s.wts[n * s.M + m] : 1.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = s.wts ? fmaf(a.get(j), w, acc[j]) : acc[j] + a.get(j);
    }
    V8<T> o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o.set(j, s.wts ? acc[j] : acc[j] * s.wconst);
    o.store(out + nv * ldo + cg * 8);
  }
}

// fuse_fwd<NORM> with the source count MM known at compile time: the MM feature loads of an item are issued
// together (the runtime-M loop waited a memory latency per source), and since the grid stride is a multiple of
// C / 8 a thread's channel group never changes, so the sources' statistics are loaded once per sample instead
// of once per item.  Same operations in the same order as fuse_fwd<NORM>: bitwise equal.
template <typename T, int MM>
__global__ void fuse_norm_fwd_m(FuseSrc s, T* __restrict__ out, int ldo, long long V, int N, int C) {
  const int C8 = C >> 3;
  const int total = N * (int)V * C8;   // < 2^31 (host check): 32-bit index math
  const int stride = gridDim.x * blockDim.x;   // a multiple of C8 (host check)
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int cg = i % C8;
  int cur_n = -1;
  float mu[MM][8], rs[MM][8];
  for (; i < total; i += stride) {
    const long long nv = i / C8;
    const int n = (int)(nv / (int)V);
    V8<T> a[MM];
#pragma unroll
    for (int m = 0; m < MM; ++m) a[m].load(reinterpret_cast<const T*>(s.p[m]) + nv * s.ld[m] + cg * 8);
    if (n != cur_n) {
#pragma unroll
      for (int m = 0; m < MM; ++m) {
        load8f(s.mean[m] + n * C + cg * 8, mu[m]);
        load8f(s.rstd[m] + n * C + cg * 8, rs[m]);
      }
      cur_n = n;
    }
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
    for (int m = 0; m < MM; ++m) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float h = (a[m].get(j) - mu[m][j]) * rs[m][j];
        a[m].set(j, h > 0.f ? h : 0.f);
      }
      const float w = s.wts ? s.wts[n * s.M + m] : 1.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = s.wts ? fmaf(a[m].get(j), w, acc[j]) : acc[j] + a[m].get(j);
    }
    V8<T> o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o.set(j, s.wts ? acc[j] : acc[j] * s.wconst);
    o.store(out + nv * ldo + cg * 8);
  }
}

// dots[n][m] partial: sum_{v,c} dfused[n,v,c] * src_m[n,v,c]
template <typename T>
__global__ void fuse_dot_partial(FuseSrc s, const T* __restrict__ dfused, int ldd, long long V, int C, long long vpc,
                                 float* __restrict__ part) {
  const int n = blockIdx.y, chunk = blockIdx.x, nchunk = gridDim.x;
  const int C8 = C >> 3;
  const int tid = threadIdx.x;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  const long long v0 = (long long)chunk * vpc;
  long long v1 = v0 + vpc;
  if (v1 > V) v1 = V;
  const long long e0 = v0 * C8, e1 = v1 * C8;
  for (long long e = e0 + tid; e < e1; e += 256) {
    const long long v = e / C8;
    const int cg = (int)(e - v * C8);
    const long long nv = (long long)n * V + v;
    V8<T> d;
    d.load(dfused + nv * ldd + cg * 8);
    for (int m = 0; m < s.M; ++m) {
      V8<T> a;
      a.load(reinterpret_cast<const T*>(s.p[m]) + nv * s.ld[m] + cg * 8);
      float t = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) t = fmaf(a.get(j), d.get(j), t);
      acc[m] += t;
    }
  }
  __shared__ float red[4][4];
  const int lane = tid & 63, wave = tid >> 6;
  for (int m = 0; m < s.M; ++m) {
    float w = wave_sum(acc[m]);
    if (lane == 0) red[m][wave] = w;
  }
  __syncthreads();
  if (tid < s.M) part[((long long)n * nchunk + chunk) * 4 + tid] = red[tid][0] + red[tid][1] + red[tid][2] + red[tid][3];
}

// ---------------------------------------------------- attention gate (SE)
// pooled [N][MC] -> h = relu(W1 pooled + b1) [N][Hd] -> logits = W2 h + b2 [N][M] -> w = softmax
__global__ void attn_gate_fwd(const float* __restrict__ pooled, const float* __restrict__ W1,
                              const float* __restrict__ b1, const float* __restrict__ W2, const float* __restrict__ b2,
                              float* __restrict__ hbuf, float* __restrict__ wts, int MC, int Hd, int M) {
  const int n = blockIdx.x;
  extern __shared__ float sh[];
  float* h = sh;  // Hd
  for (int k = threadIdx.x; k < Hd; k += blockDim.x) {
    float a = 0.f;
    for (int i = 0; i < MC; ++i) a = fmaf(W1[(long long)k * MC + i], pooled[(long long)n * MC + i], a);
    a += b1[k];
    a = a > 0.f ? a : 0.f;
    h[k] = a;
    hbuf[(long long)n * Hd + k] = a;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float lg[4];
    float mx = -INFINITY;
    for (int m = 0; m < M; ++m) {
      float a = 0.f;
      for (int k = 0; k < Hd; ++k) a = fmaf(W2[m * Hd + k], h[k], a);
      lg[m] = a + b2[m];
      mx = fmaxf(mx, lg[m]);
    }
    float se = 0.f;
    for (int m = 0; m < M; ++m) {
      lg[m] = expf(lg[m] - mx);
      se += lg[m];
    }
    for (int m = 0; m < M; ++m) wts[n * M + m] = lg[m] / se;
  }
}

// Backward of the gate for all N (one block): inputs dots part -> dw[n][m];
// writes beta[n][MC] = dpooled / V and the Linear gradients (accumulated).
__global__ void attn_gate_bwd(const float* __restrict__ dot_part, int nchunk, const float* __restrict__ pooled,
                              const float* __restrict__ W1, const float* __restrict__ W2,
                              const float* __restrict__ hbuf, const float* __restrict__ wts, float* __restrict__ beta,
                              float* __restrict__ gW1, float* __restrict__ gb1, float* __restrict__ gW2,
                              float* __restrict__ gb2, int N, int MC, int Hd, int M, long long V, int accumulate) {
  extern __shared__ float sh[];
  float* dlog = sh;              // N*M
  float* dh = sh + N * M;        // N*Hd
  const int tid = threadIdx.x;
  if (tid < N * M) {
    const int n = tid / M, m = tid % M;
    // dw for (n, *) in fixed order
    float dw[4];
    float s = 0.f;
    for (int mm = 0; mm < M; ++mm) {
      float a = 0.f;
      for (int k = 0; k < nchunk; ++k) a += dot_part[((long long)n * nchunk + k) * 4 + mm];
      dw[mm] = a;
      s += wts[n * M + mm] * a;
    }
    dlog[tid] = wts[n * M + m] * (dw[m] - s);
  }
  __syncthreads();
  for (int e = tid; e < N * Hd; e += blockDim.x) {
    const int n = e / Hd, k = e % Hd;
    float a = 0.f;
    for (int m = 0; m < M; ++m) a = fmaf(W2[m * Hd + k], dlog[n * M + m], a);
    dh[e] = hbuf[e] > 0.f ? a : 0.f;
  }
  __syncthreads();
  // Linear2 grads
  for (int e = tid; e < M * Hd; e += blockDim.x) {
    const int m = e / Hd, k = e % Hd;
    float a = 0.f;
    for (int n = 0; n < N; ++n) a = fmaf(dlog[n * M + m], hbuf[n * Hd + k], a);
    gW2[e] = accumulate ? gW2[e] + a : a;
  }
  for (int m = tid; m < M; m += blockDim.x) {
    float a = 0.f;
    for (int n = 0; n < N; ++n) a += dlog[n * M + m];
    gb2[m] = accumulate ? gb2[m] + a : a;
  }
  // Linear1 grads and dpooled
  for (long long e = tid; e < (long long)Hd * MC; e += blockDim.x) {
    const int k = (int)(e / MC), i = (int)(e % MC);
    float a = 0.f;
    for (int n = 0; n < N; ++n) a = fmaf(dh[n * Hd + k], pooled[(long long)n * MC + i], a);
    gW1[e] = accumulate ? gW1[e] + a : a;
  }
  for (int k = tid; k < Hd; k += blockDim.x) {
    float a = 0.f;
    for (int n = 0; n < N; ++n) a += dh[n * Hd + k];
    gb1[k] = accumulate ? gb1[k] + a : a;
  }
  const float invV = 1.f / (float)V;
  for (long long e = tid; e < (long long)N * MC; e += blockDim.x) {
    const int n = (int)(e / MC), i = (int)(e % MC);
    float a = 0.f;
    for (int k = 0; k < Hd; ++k) a = fmaf(W1[(long long)k * MC + i], dh[n * Hd + k], a);
    beta[e] = a * invV;
  }
}

// Kernels with a 32-bit grid-stride index (maxpool2_fwd, fuse_fwd) step i by up to 8192 * 256 = 2^21: the
// item count must stay that far below INT_MAX so the last i += stride cannot wrap negative.
constexpr long long kGridStrideMax = 2147483647LL - 8192LL * 256;

int grid_for(long long total) {
  long long b = (total + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (int)b;
}

int knob_small_v() {   // read per call (A/B runs and tests flip it in-process)
  const char* e = getenv("MMSEG_IN_SMALL_V");
  return e ? atoi(e) : 4096;
}



// at least 256 chunks per sample (down to 2 voxels per thread): the 48^3 / 24^3 levels otherwise ran 108..432
// blocks of 16 voxels per thread, latency-bound (128 / 512 measured within noise, r03u)
int knob_in_minch() { return 256; }

int chunks_for(long long V, int C, long long* vpc) {
  // reduction passes: ~16 voxels per thread (lanes_v = 256 / C8 voxel lanes), at most 1024 chunks
  const int lanes_v = 256 / (C >> 3);
  long long want = (long long)lanes_v * 16;
  long long nch = (V + want - 1) / want;
  const long long minch = std::min<long long>(knob_in_minch(), V / (2LL * lanes_v));
  if (nch < minch) nch = minch;
  if (nch > 1024) nch = 1024;
  if (nch < 1) nch = 1;
  *vpc = (V + nch - 1) / nch;
  return (int)((V + *vpc - 1) / *vpc);
}

int apply_chunks(long long V, int C, int* vpc) {
  // elementwise passes: 2 x UNR voxels per thread
  const int lanes_v = 256 / (C >> 3);
  long long want = (long long)lanes_v * 2 * UNR;
  long long nch = (V + want - 1) / want;
  const long long minch = std::min<long long>(knob_in_minch(), V / lanes_v);
  if (nch < minch) nch = minch;
  if (nch < 1) nch = 1;
  *vpc = (int)((V + nch - 1) / nch);
  return (int)((V + *vpc - 1) / *vpc);
}

}  // namespace

extern "C" {

// Workspace (floats) the stats / bwd-reduce kernels need for N samples.
long long mmseg_instnorm_ws_floats(int N, long long V, int C) {
  long long vpc;
  int nch = chunks_for(V, C, &vpc);
  return (long long)N * nch * C * 2 + (long long)N * C * 2;
}

// mean[n*mean_ld + c], rstd[n*C + c] (rstd may be null: channel means only)
int mmseg_instnorm_stats(const void* x, int ldx, int N, long long V, int C, float eps, float* mean, int mean_ld,
                         float* rstd, float* ws, int dtype, void* stream) {
  MMSEG_REQUIRE(C % 8 == 0 && C <= 2048, "instnorm: C=%d must be a multiple of 8", C);
  MMSEG_REQUIRE(V * ldx < (1LL << 31), "instnorm: per-sample extent must fit int32");
  long long vpc;
  const int nch = chunks_for(V, C, &vpc);
  hipStream_t s = (hipStream_t)stream;
  dim3 grid(nch, N);
  if (dtype == MMSEG_BF16) {
    MMSEG_LAUNCH(in_stats_partial<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)x, ldx, (int)V, C, (int)vpc,
                       ws);
    MMSEG_LAUNCH(in_stats_finalize<bf16_t>, dim3(N * C), dim3(256), 0, s, (const bf16_t*)x, ldx,
                       V, N, C, nch, vpc, ws, eps, mean, mean_ld, rstd);
  } else {
    MMSEG_LAUNCH(in_stats_partial<float>, grid, dim3(256), 0, s, (const float*)x, ldx, (int)V, C, (int)vpc, ws);
    MMSEG_LAUNCH(in_stats_finalize<float>, dim3(N * C), dim3(256), 0, s, (const float*)x, ldx, V,
                       N, C, nch, vpc, ws, eps, mean, mean_ld, rstd);
  }
  return mmseg::check_launch("instnorm_stats");
}

// mean / rstd from the per-brick partials of mmseg_conv_gemm_stats (nb bricks of cnt voxels per sample).
int mmseg_instnorm_stats_bricks(const float* part, int N, int C, int nb, int cnt, float eps, float* mean, int mean_ld,
                                float* rstd, void* stream) {
  MMSEG_REQUIRE(nb >= 1 && cnt >= 1, "instnorm_stats_bricks: nb, cnt >= 1");
  MMSEG_LAUNCH(in_stats_from_bricks, dim3(ceil_div(N * C, 4)), dim3(256), 0, (hipStream_t)stream, part, N, C,
                     nb, cnt, eps, mean, mean_ld, rstd);
  return mmseg::check_launch("instnorm_stats_bricks");
}

int mmseg_instnorm_apply(const void* x, int ldx, void* y, int ldy, int N, long long V, int C, const float* mean,
                         const float* rstd, int relu, int dtype, void* stream);
int mmseg_instnorm_stats(const void* x, int ldx, int N, long long V, int C, float eps, float* mean, int mean_ld,
                         float* rstd, float* ws, int dtype, void* stream);
int mmseg_instnorm_bwd(const void* x, int ldx, const float* mean, const float* rstd, const void* p1, int ld1,
                       float scale1, const float* alpha1, int alpha_stride, const float* beta, int beta_stride,
                       const void* pool_dy, int pool_ld, const uint8_t* pool_idx, void* dx, int lddx, int N, int D,
                       int H, int W, int C, int relu, float* ws, int dtype, void* stream);

int mmseg_instnorm_fwd(const void* x, int ldx, void* y, int ldy, int N, long long V, int C, float eps, float* mean,
                       int mean_ld, float* rstd, int relu, float* ws, int dtype, void* stream) {
  MMSEG_REQUIRE(C % 8 == 0 && C <= 2048, "instnorm_fwd: C=%d must be a multiple of 8", C);
  if (V > knob_small_v()) {
    if (mmseg_instnorm_stats(x, ldx, N, V, C, eps, mean, mean_ld, rstd, ws, dtype, stream)) return 1;
    MMSEG_REQUIRE(mean_ld == C, "instnorm_fwd: the apply pass reads mean with ld = C");
    return mmseg_instnorm_apply(x, ldx, y, ldy, N, V, C, mean, rstd, relu, dtype, stream);
  }
  MMSEG_REQUIRE(V * (ldx > ldy ? ldx : ldy) < (1LL << 31), "instnorm_fwd: per-sample extent must fit int32");
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(C / 8, N);
  auto run = [&](auto tag, auto relu_c) {
    using T = decltype(tag);
    constexpr bool R = decltype(relu_c)::value;
    if (V <= SMALL_T)
      MMSEG_LAUNCH((in_small_fwd_r<T, R, 1>), grid, dim3(SMALL_T), 0, s, (const T*)x, ldx, (T*)y, ldy, (int)V, C,
                         eps, mean, mean_ld, rstd);
    else if (V <= 8 * SMALL_T)
      MMSEG_LAUNCH((in_small_fwd_r<T, R, 8>), grid, dim3(SMALL_T), 0, s, (const T*)x, ldx, (T*)y, ldy, (int)V, C,
                         eps, mean, mean_ld, rstd);
    else
      MMSEG_LAUNCH((in_small_fwd<T, R>), grid, dim3(SMALL_T), 0, s, (const T*)x, ldx, (T*)y, ldy, (int)V, C, eps,
                         mean, mean_ld, rstd);
  };
  if (dtype == MMSEG_BF16) {
    if (relu) run(bf16_t{}, std::true_type{});
    else run(bf16_t{}, std::false_type{});
  } else {
    if (relu) run(float{}, std::true_type{});
    else run(float{}, std::false_type{});
  }
  return mmseg::check_launch("instnorm_fwd");
}

int mmseg_instnorm_relu_fwd(const void* x, int ldx, void* y, int ldy, int N, long long V, int C, const float* mean,
                            const float* rstd, int dtype, void* stream) {
  return mmseg_instnorm_apply(x, ldx, y, ldy, N, V, C, mean, rstd, 1, dtype, stream);
}

int mmseg_instnorm_apply(const void* x, int ldx, void* y, int ldy, int N, long long V, int C, const float* mean,
                         const float* rstd, int relu, int dtype, void* stream) {
  MMSEG_REQUIRE(C % 8 == 0 && C <= 2048, "instnorm_apply: C=%d must be a multiple of 8", C);
  MMSEG_REQUIRE(V * (ldx > ldy ? ldx : ldy) < (1LL << 31), "instnorm_apply: per-sample extent must fit int32");
  hipStream_t s = (hipStream_t)stream;
  int vpc;
  const dim3 grid(apply_chunks(V, C, &vpc), N);
  if (dtype == MMSEG_BF16) {
    if (relu)
      MMSEG_LAUNCH((in_relu_apply<bf16_t, true>), grid, dim3(256), 0, s, (const bf16_t*)x, ldx, (bf16_t*)y, ldy,
                         (int)V, C, vpc, mean, rstd);
    else
      MMSEG_LAUNCH((in_relu_apply<bf16_t, false>), grid, dim3(256), 0, s, (const bf16_t*)x, ldx, (bf16_t*)y,
                         ldy, (int)V, C, vpc, mean, rstd);
  } else {
    if (relu)
      MMSEG_LAUNCH((in_relu_apply<float, true>), grid, dim3(256), 0, s, (const float*)x, ldx, (float*)y, ldy,
                         (int)V, C, vpc, mean, rstd);
    else
      MMSEG_LAUNCH((in_relu_apply<float, false>), grid, dim3(256), 0, s, (const float*)x, ldx, (float*)y, ldy,
                         (int)V, C, vpc, mean, rstd);
  }
  return mmseg::check_launch("instnorm_apply");
}

// dy sources: see DySrc.  Any of p1 / beta / pool_dy may be null.
int mmseg_instnorm_relu_bwd(const void* x, int ldx, const float* mean, const float* rstd, const void* p1, int ld1,
                            float scale1, const float* alpha1, int alpha_stride, const float* beta, int beta_stride,
                            const void* pool_dy, int pool_ld, const uint8_t* pool_idx, void* dx, int lddx, int N,
                            int D, int H, int W, int C, float* ws, int dtype, void* stream) {
  return mmseg_instnorm_bwd(x, ldx, mean, rstd, p1, ld1, scale1, alpha1, alpha_stride, beta, beta_stride, pool_dy,
                            pool_ld, pool_idx, dx, lddx, N, D, H, W, C, 1, ws, dtype, stream);
}

int mmseg_instnorm_bwd_part(const void* x, int ldx, const float* mean, const float* rstd, const void* p1, int ld1,
                            float scale1, const float* alpha1, int alpha_stride, const float* beta, int beta_stride,
                            const void* pool_dy, int pool_ld, const uint8_t* pool_idx, void* dx, int lddx, int N,
                            int D, int H, int W, int C, int relu, const float* part_in, int nchunk_in, float* ws,
                            int dtype, void* stream);
int instnorm_bwd_impl(const void* x, int ldx, const float* mean, const float* rstd, const void* p1, int ld1,
                      float scale1, const float* alpha1, int alpha_stride, const float* beta, int beta_stride,
                      const void* pool_dy, int pool_ld, const uint8_t* pool_idx, void* dx, int lddx, int N, int D,
                      int H, int W, int C, int relu, const float* part_in, int nchunk_in, float* ws, int dtype,
                      void* stream, int p1_nmod, float slope = 0.f, int Cw = 0);

// The InstanceNorm + ReLU backward of G modality encoders' level outputs at once (N = G x n samples of one
// combined pre-norm tensor / statistics / pooled gradient): every sample reads the fused level's gradient p1 of
// its own sample index modulo p1_nmod = n -- once per fused sample for all G modalities (reference
// dual_encoder.py:193-195 mean / 184-186 add fusion backward, unet.py:34-35 InstanceNorm + ReLU).
int mmseg_instnorm_relu_bwd_group(const void* x, int ldx, const float* mean, const float* rstd, const void* p1,
                                  int ld1, float scale1, int p1_nmod, const void* pool_dy, int pool_ld,
                                  const uint8_t* pool_idx, void* dx, int lddx, int N, int D, int H, int W, int C,
                                  float* ws, int dtype, void* stream) {
  MMSEG_REQUIRE(p1_nmod >= 1 && N % p1_nmod == 0, "instnorm_relu_bwd_group: N=%d must be a multiple of p1_nmod=%d",
                N, p1_nmod);
  return instnorm_bwd_impl(x, ldx, mean, rstd, p1, ld1, scale1, nullptr, 0, nullptr, 0, pool_dy, pool_ld, pool_idx,
                           dx, lddx, N, D, H, W, C, 1, nullptr, 0, ws, dtype, stream, p1_nmod);
}

// The InstanceNorm backward (no affine) with the activation after the norm folded in (act 0 none, 1 ReLU, 2
// LeakyReLU(slope); g: the gradient of the activation's OUTPUT), dy = g: SwinUNETR's UnetResBlock norms (MONAI
// get_norm_layer("instance") + LeakyReLU(0.01) for conv1's, none for conv2 / conv3's, whose LeakyReLU follows the
// residual sum -- mmseg_lrelu_bwd_in_part).  part / nchunk: partial sums a producer of g emitted (finalize + apply
// only), or null.  Cw: dx's channels [C, Cw) are written as zeros (whole-row writes at pitch lddx > C) on the
// partial / apply path (V > the small-volume bound).
int mmseg_instnorm_act_bwd(const void* x, int ldx, const float* mean, const float* rstd, const void* g, int ldg,
                           void* dx, int lddx, int N, int D, int H, int W, int C, int Cw, int act, float slope,
                           const float* part, int nchunk, float* ws, int dtype, void* stream) {
  return instnorm_bwd_impl(x, ldx, mean, rstd, g, ldg, 1.f, nullptr, 0, nullptr, 0, nullptr, 0, nullptr, dx, lddx, N,
                           D, H, W, C, act, part, nchunk, ws, dtype, stream, 0, slope, Cw);
}

int mmseg_instnorm_part_chunks(long long V, int C) {
  long long vpc;
  return (C % 8 == 0 && C <= 2048 && V > 0) ? chunks_for(V, C, &vpc) : 0;
}

int mmseg_lrelu_bwd_in_part(const void* y, int ldy, const void* dy, int lddy, void* g, int ldg, float slope,
                            const void* xa, int lda, const float* ma, const float* ra, float* pa, const void* xb,
                            int ldb, const float* mb, const float* rb, float* pb, int N, long long V, int C, int Cw,
                            int dtype, void* stream) {
  MMSEG_REQUIRE(C % 8 == 0 && C <= 2048 && V > 0, "lrelu_bwd_in_part: C=%d must be a multiple of 8", C);
  MMSEG_REQUIRE(Cw % 8 == 0 && Cw >= C && Cw <= 2 * C && Cw <= ldg, "lrelu_bwd_in_part: C <= Cw <= min(2 C, ldg)");
  const int npad = (Cw - C) / 8;
  MMSEG_REQUIRE(y && dy && g && xa && ma && ra && pa, "lrelu_bwd_in_part: null operand");
  MMSEG_REQUIRE(!xb || (mb && rb && pb), "lrelu_bwd_in_part: xb needs its statistics and partial buffer");
  const int ldmax = std::max(std::max(ldy, lddy), std::max(std::max(ldg, lda), xb ? ldb : 0));
  MMSEG_REQUIRE(V * ldmax < (1LL << 31), "lrelu_bwd_in_part: per-sample extent must fit int32");
  MMSEG_REQUIRE(ldy % 8 == 0 && lddy % 8 == 0 && ldg % 8 == 0 && lda % 8 == 0 && (!xb || ldb % 8 == 0),
                "lrelu_bwd_in_part: pitches must be multiples of 8");
  long long vpc;
  const int nch = chunks_for(V, C, &vpc);
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(nch, N);
  auto run = [&](auto tag, auto zp) {
    using T = decltype(tag);
    constexpr bool Z = decltype(zp)::value;
    if (xb)
      MMSEG_LAUNCH((lrelu_bwd_in_partial<T, 2, Z>), grid, dim3(256), 0, s, (const T*)y, ldy, (const T*)dy, lddy, (T*)g,
                   ldg, slope, (const T*)xa, lda, ma, ra, pa, (const T*)xb, ldb, mb, rb, pb, (int)V, C, (int)vpc,
                   npad);
    else
      MMSEG_LAUNCH((lrelu_bwd_in_partial<T, 1, Z>), grid, dim3(256), 0, s, (const T*)y, ldy, (const T*)dy, lddy, (T*)g,
                   ldg, slope, (const T*)xa, lda, ma, ra, pa, (const T*)nullptr, 0, nullptr, nullptr, nullptr, (int)V,
                   C, (int)vpc, npad);
  };
  auto zrun = [&](auto tag) {
    if (npad) run(tag, std::true_type{});
    else run(tag, std::false_type{});
  };
  if (dtype == MMSEG_BF16) zrun(bf16_t{});
  else zrun(float{});
  return mmseg::check_launch("lrelu_bwd_in_part");
}

int mmseg_instnorm_bwd(const void* x, int ldx, const float* mean, const float* rstd, const void* p1, int ld1,
                            float scale1, const float* alpha1, int alpha_stride, const float* beta, int beta_stride,
                            const void* pool_dy, int pool_ld, const uint8_t* pool_idx, void* dx, int lddx, int N,
                            int D, int H, int W, int C, int relu, float* ws, int dtype, void* stream) {
  return mmseg_instnorm_bwd_part(x, ldx, mean, rstd, p1, ld1, scale1, alpha1, alpha_stride, beta, beta_stride, pool_dy,
                                 pool_ld, pool_idx, dx, lddx, N, D, H, W, C, relu, nullptr, 0, ws, dtype, stream);
}

// mmseg_instnorm_bwd whose partial sums (g, g * xhat per chunk, [N][nchunk_in][C][2]) a producer of dy already
// emitted (the fused head + loss backward, mmseg_head_loss_bwd_in): the partial pass is skipped.
int mmseg_instnorm_bwd_part(const void* x, int ldx, const float* mean, const float* rstd, const void* p1, int ld1,
                            float scale1, const float* alpha1, int alpha_stride, const float* beta, int beta_stride,
                            const void* pool_dy, int pool_ld, const uint8_t* pool_idx, void* dx, int lddx, int N,
                            int D, int H, int W, int C, int relu, const float* part_in, int nchunk_in, float* ws,
                            int dtype, void* stream) {
  return instnorm_bwd_impl(x, ldx, mean, rstd, p1, ld1, scale1, alpha1, alpha_stride, beta, beta_stride, pool_dy,
                           pool_ld, pool_idx, dx, lddx, N, D, H, W, C, relu, part_in, nchunk_in, ws, dtype, stream, 0);
}

int instnorm_bwd_impl(const void* x, int ldx, const float* mean, const float* rstd, const void* p1, int ld1,
                      float scale1, const float* alpha1, int alpha_stride, const float* beta, int beta_stride,
                      const void* pool_dy, int pool_ld, const uint8_t* pool_idx, void* dx, int lddx, int N, int D,
                      int H, int W, int C, int relu, const float* part_in, int nchunk_in, float* ws, int dtype,
                      void* stream, int p1_nmod, float slope, int Cw) {
  MMSEG_REQUIRE(relu >= 0 && relu <= 2, "instnorm_bwd: activation %d (0 none, 1 ReLU, 2 LeakyReLU)", relu);
  if (Cw == 0) Cw = C;
  MMSEG_REQUIRE(Cw % 8 == 0 && Cw >= C && Cw <= 2 * C && Cw <= lddx,
                "instnorm_bwd: write extent Cw=%d outside [C, min(2 C, lddx)] or not a multiple of 8", Cw);
  const int npad = (Cw - C) / 8;
  MMSEG_REQUIRE(C % 8 == 0 && C <= 2048, "instnorm_bwd: C=%d must be a multiple of 8 and <= 2048", C);
  MMSEG_REQUIRE(!part_in || nchunk_in > 0, "instnorm_bwd: given partials need their chunk count");
  MMSEG_REQUIRE(!pool_dy || ((D | H | W) & 1) == 0, "instnorm_bwd: pooled gather needs even dims");
  const long long V = (long long)D * H * W;
  MMSEG_REQUIRE(V * (ldx > lddx ? ldx : lddx) < (1LL << 31) && V * (ld1 > pool_ld ? ld1 : pool_ld) < (1LL << 31),
                "instnorm_bwd: per-sample extent must fit int32");
  long long vpc;
  const int nch = chunks_for(V, C, &vpc);
  int avpc;
  const int anch = apply_chunks(V, C, &avpc);
  DySrc src{p1, ld1, scale1, alpha1, alpha_stride, beta, beta_stride, pool_dy, pool_ld, pool_idx, p1_nmod, slope};
  hipStream_t s = (hipStream_t)stream;
  float* part = ws;
  float* coef = ws + (long long)N * nch * C * 2;
  dim3 grid(nch, N), agrid(anch, N);
  if (p1_nmod > 0 && N / p1_nmod > 1) {   // modality groups sharing a p1 sample: chunk-major grids (DySrc::gsplit)
    src.gsplit = N / p1_nmod;
    grid = dim3(nch * src.gsplit, p1_nmod);
    agrid = dim3(anch * src.gsplit, p1_nmod);
  }
  const bool small = V <= knob_small_v() && !part_in;
  if (part_in) coef = ws;
  auto run = [&](auto tag, auto act_c) {
    using T = decltype(tag);
    constexpr int R = decltype(act_c)::value;
    if (part_in) {
      MMSEG_LAUNCH(in_bwd_finalize, dim3(N * C), dim3(256), 0, s, part_in, N, C, nchunk_in, V, coef);
      if (npad)
        MMSEG_LAUNCH((in_bwd_apply<T, R, true>), agrid, dim3(256), 0, s, (const T*)x, ldx, mean, rstd, src, coef,
                           (T*)dx, lddx, (int)V, C, D, H, W, avpc, npad);
      else
        MMSEG_LAUNCH((in_bwd_apply<T, R>), agrid, dim3(256), 0, s, (const T*)x, ldx, mean, rstd, src, coef,
                           (T*)dx, lddx, (int)V, C, D, H, W, avpc, 0);
      return;
    }
    if (small) {
      if (V <= SMALL_T)
        MMSEG_LAUNCH((in_small_bwd_r<T, R, 1>), dim3(C / 8, N), dim3(SMALL_T), 0, s, (const T*)x, ldx, mean, rstd,
                           src, (T*)dx, lddx, (int)V, C, D, H, W);
      else if (V <= 8 * SMALL_T)
        MMSEG_LAUNCH((in_small_bwd_r<T, R, 8>), dim3(C / 8, N), dim3(SMALL_T), 0, s, (const T*)x, ldx, mean, rstd,
                           src, (T*)dx, lddx, (int)V, C, D, H, W);
      else
        MMSEG_LAUNCH((in_small_bwd<T, R>), dim3(C / 8, N), dim3(SMALL_T), 0, s, (const T*)x, ldx, mean, rstd, src,
                           (T*)dx, lddx, (int)V, C, D, H, W);
      return;
    }
    MMSEG_LAUNCH((in_bwd_partial<T, R>), grid, dim3(256), 0, s, (const T*)x, ldx, mean, rstd, src, (int)V, C, D,
                       H, W, (int)vpc, part);
    MMSEG_LAUNCH(in_bwd_finalize, dim3(N * C), dim3(256), 0, s, part, N, C, nch, V, coef);
    if (npad)
      MMSEG_LAUNCH((in_bwd_apply<T, R, true>), agrid, dim3(256), 0, s, (const T*)x, ldx, mean, rstd, src, coef,
                         (T*)dx, lddx, (int)V, C, D, H, W, avpc, npad);
    else
      MMSEG_LAUNCH((in_bwd_apply<T, R>), agrid, dim3(256), 0, s, (const T*)x, ldx, mean, rstd, src, coef, (T*)dx,
                         lddx, (int)V, C, D, H, W, avpc, 0);
  };
  auto act = [&](auto tag) {
    if (relu == 2) run(tag, std::integral_constant<int, 2>{});
    else if (relu == 1) run(tag, std::integral_constant<int, 1>{});
    else run(tag, std::integral_constant<int, 0>{});
  };
  if (dtype == MMSEG_BF16) act(bf16_t{});
  else act(float{});
  return mmseg::check_launch("instnorm_relu_bwd");
}

// The first half of mmseg_instnorm_bwd for dy = p1 (scale 1): the finalised coefficients coef [N][C][2] =
// (mean g, mean g xhat), from the partials a producer of dy emitted (part_in, nchunk_in) or from the partial pass
// (part_in null; ws: mmseg_instnorm_ws_floats).  The apply half then runs inside the norm's only consumer
// (mmseg_stem_wgrad_inb), which never writes the input gradient.
int mmseg_instnorm_bwd_coef(const void* x, int ldx, const float* mean, const float* rstd, const void* p1, int ld1,
                            int N, int D, int H, int W, int C, int relu, const float* part_in, int nchunk_in,
                            float* coef, float* ws, int dtype, void* stream) {
  MMSEG_REQUIRE(C % 8 == 0 && C <= 2048 && p1 && coef, "instnorm_bwd_coef: C=%d must be a multiple of 8", C);
  const long long V = (long long)D * H * W;
  MMSEG_REQUIRE(V * (ldx > ld1 ? ldx : ld1) < (1LL << 31), "instnorm_bwd_coef: per-sample extent must fit int32");
  hipStream_t s = (hipStream_t)stream;
  if (!part_in) {
    long long vpc;
    const int nch = chunks_for(V, C, &vpc);
    DySrc src{p1, ld1, 1.f, nullptr, 0, nullptr, 0, nullptr, 0, nullptr};
    const dim3 grid(nch, N);
    auto run = [&](auto tag, auto act_c) {
      using T = decltype(tag);
      constexpr int R = decltype(act_c)::value;
      MMSEG_LAUNCH((in_bwd_partial<T, R>), grid, dim3(256), 0, s, (const T*)x, ldx, mean, rstd, src, (int)V, C,
                         D, H, W, (int)vpc, ws);
    };
    if (dtype == MMSEG_BF16) {
      if (relu) run(bf16_t{}, std::integral_constant<int, 1>{});
      else run(bf16_t{}, std::integral_constant<int, 0>{});
    } else {
      if (relu) run(float{}, std::integral_constant<int, 1>{});
      else run(float{}, std::integral_constant<int, 0>{});
    }
    part_in = ws;
    nchunk_in = nch;
  }
  MMSEG_LAUNCH(in_bwd_finalize, dim3(N * C), dim3(256), 0, s, part_in, N, C, nchunk_in, V, coef);
  return mmseg::check_launch("instnorm_bwd_coef");
}

int mmseg_maxpool2_fwd(const void* x, int ldx, void* y, int ldy, uint8_t* idx, int N, int D, int H, int W, int C,
                       int dtype, void* stream) {
  MMSEG_REQUIRE(C % 8 == 0 && ((D | H | W) & 1) == 0, "maxpool2: C%%8==0 and even dims required");
  MMSEG_REQUIRE((long long)N * (D / 2) * (H / 2) * (W / 2) * (C / 8) <= kGridStrideMax, "maxpool2: too many items");
  hipStream_t s = (hipStream_t)stream;
  const int grid = grid_for((long long)N * (D / 2) * (H / 2) * (W / 2) * (C / 8));
  if (dtype == MMSEG_BF16)
    MMSEG_LAUNCH(maxpool2_fwd<bf16_t>, dim3(grid), dim3(256), 0, s, (const bf16_t*)x, ldx, (bf16_t*)y, ldy, idx,
                       N, D, H, W, C, (const float*)nullptr, (const float*)nullptr);
  else
    MMSEG_LAUNCH(maxpool2_fwd<float>, dim3(grid), dim3(256), 0, s, (const float*)x, ldx, (float*)y, ldy, idx, N,
                       D, H, W, C, (const float*)nullptr, (const float*)nullptr);
  return mmseg::check_launch("maxpool2_fwd");
}

// mmseg_maxpool2_fwd over relu((x - mean) * rstd) (x pre-norm, mean / rstd [N][C]): equal to pooling the
// materialised InstanceNorm + ReLU output.
int mmseg_maxpool2_norm_fwd(const void* x, int ldx, const float* mean, const float* rstd, void* y, int ldy,
                            uint8_t* idx, int N, int D, int H, int W, int C, int dtype, void* stream) {
  MMSEG_REQUIRE(C % 8 == 0 && ((D | H | W) & 1) == 0, "maxpool2: C%%8==0 and even dims required");
  MMSEG_REQUIRE((long long)N * (D / 2) * (H / 2) * (W / 2) * (C / 8) <= kGridStrideMax, "maxpool2: too many items");
  hipStream_t s = (hipStream_t)stream;
  const int grid = grid_for((long long)N * (D / 2) * (H / 2) * (W / 2) * (C / 8));
  if (dtype == MMSEG_BF16)
    MMSEG_LAUNCH((maxpool2_fwd<bf16_t, true>), dim3(grid), dim3(256), 0, s, (const bf16_t*)x, ldx, (bf16_t*)y,
                       ldy, idx, N, D, H, W, C, mean, rstd);
  else
    MMSEG_LAUNCH((maxpool2_fwd<float, true>), dim3(grid), dim3(256), 0, s, (const float*)x, ldx, (float*)y, ldy,
                       idx, N, D, H, W, C, mean, rstd);
  return mmseg::check_launch("maxpool2_norm_fwd");
}

// mmseg_fuse_fwd over relu((src_m - mean_m) * rstd_m) (pre-norm sources, statistics [N][C] per source)
int mmseg_fuse_norm_fwd(const void* const* srcs, const int* lds, const float* const* means, const float* const* rstds,
                        int M, float wconst, const float* wts, void* out, int ldo, int N, long long V, int C,
                        int dtype, void* stream) {
  MMSEG_REQUIRE(M >= 1 && M <= 4 && C % 8 == 0, "fuse: 1 <= M <= 4 and C%%8==0");
  MMSEG_REQUIRE((long long)N * V * (C / 8) <= kGridStrideMax, "fuse: too many items");
  FuseSrc s{};
  for (int m = 0; m < M; ++m) {
    s.p[m] = srcs[m];
    s.ld[m] = lds[m];
    s.mean[m] = means[m];
    s.rstd[m] = rstds[m];
  }
  s.M = M;
  s.wconst = wconst;
  s.wts = wts;
  hipStream_t st = (hipStream_t)stream;
  const int grid = grid_for((long long)N * V * (C / 8));
  // compile-time M for 2 and 3 sources (M = 4 spilled and stays runtime-M)
  const bool cm = M >= 2 && ((long long)grid * 256) % (C / 8) == 0;
  auto run = [&](auto tag) {
    using T = decltype(tag);
    if (cm && M == 2)
      MMSEG_LAUNCH((fuse_norm_fwd_m<T, 2>), dim3(grid), dim3(256), 0, st, s, (T*)out, ldo, V, N, C);
    else if (cm && M == 3)
      MMSEG_LAUNCH((fuse_norm_fwd_m<T, 3>), dim3(grid), dim3(256), 0, st, s, (T*)out, ldo, V, N, C);
    else
      MMSEG_LAUNCH((fuse_fwd<T, true>), dim3(grid), dim3(256), 0, st, s, (T*)out, ldo, V, N, C);
  };
  if (dtype == MMSEG_BF16) run(bf16_t{});
  else run(float{});
  return mmseg::check_launch("fuse_norm_fwd");
}

// out = wconst * sum_m src_m   (wts == null)   or   sum_m wts[n][m] * src_m
int mmseg_fuse_fwd(const void* const* srcs, const int* lds, int M, float wconst, const float* wts, void* out, int ldo,
                   int N, long long V, int C, int dtype, void* stream) {
  MMSEG_REQUIRE(M >= 1 && M <= 4 && C % 8 == 0, "fuse: 1 <= M <= 4 and C%%8==0");
  MMSEG_REQUIRE((long long)N * V * (C / 8) <= kGridStrideMax, "fuse: too many items");
  FuseSrc s{};
  for (int m = 0; m < M; ++m) {
    s.p[m] = srcs[m];
    s.ld[m] = lds[m];
  }
  s.M = M;
  s.wconst = wconst;
  s.wts = wts;
  hipStream_t st = (hipStream_t)stream;
  const int grid = grid_for((long long)N * V * (C / 8));
  if (dtype == MMSEG_BF16)
    MMSEG_LAUNCH(fuse_fwd<bf16_t>, dim3(grid), dim3(256), 0, st, s, (bf16_t*)out, ldo, V, N, C);
  else
    MMSEG_LAUNCH(fuse_fwd<float>, dim3(grid), dim3(256), 0, st, s, (float*)out, ldo, V, N, C);
  return mmseg::check_launch("fuse_fwd");
}

int mmseg_attn_gate_fwd(const float* pooled, const float* W1, const float* b1, const float* W2, const float* b2,
                        float* hbuf, float* wts, int N, int MC, int Hd, int M, void* stream) {
  MMSEG_REQUIRE(M <= 4, "attn gate: M <= 4");
  MMSEG_LAUNCH(attn_gate_fwd, dim3(N), dim3(256), Hd * sizeof(float), (hipStream_t)stream, pooled, W1, b1, W2,
                     b2, hbuf, wts, MC, Hd, M);
  return mmseg::check_launch("attn_gate_fwd");
}

// Backward of the attention fusion gate.  Computes dw from (dfused . src_m),
// then beta = dpooled / V (feed to instnorm_relu_bwd) and the Linear grads.
int mmseg_attn_gate_bwd(const void* const* srcs, const int* lds, int M, const void* dfused, int ldd, int N, long long V,
                        int C, const float* pooled, const float* W1, const float* W2, const float* hbuf,
                        const float* wts, float* beta, float* gW1, float* gb1, float* gW2, float* gb2, int Hd,
                        float* ws, int accumulate, int dtype, void* stream) {
  MMSEG_REQUIRE(M <= 4 && C % 8 == 0, "attn gate bwd: M <= 4");
  FuseSrc s{};
  for (int m = 0; m < M; ++m) {
    s.p[m] = srcs[m];
    s.ld[m] = lds[m];
  }
  s.M = M;
  long long want = 256 * 64;
  long long nch = (V * (C / 8) + want - 1) / want;
  if (nch > 256) nch = 256;
  long long vpc = (V + nch - 1) / nch;
  nch = (V + vpc - 1) / vpc;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == MMSEG_BF16)
    MMSEG_LAUNCH(fuse_dot_partial<bf16_t>, dim3((int)nch, N), dim3(256), 0, st, s, (const bf16_t*)dfused, ldd, V,
                       C, vpc, ws);
  else
    MMSEG_LAUNCH(fuse_dot_partial<float>, dim3((int)nch, N), dim3(256), 0, st, s, (const float*)dfused, ldd, V, C,
                       vpc, ws);
  if (mmseg::check_launch("fuse_dot_partial")) return 1;
  const int MC = M * C;
  const size_t shm = (size_t)(N * M + N * Hd) * sizeof(float);
  MMSEG_LAUNCH(attn_gate_bwd, dim3(1), dim3(256), shm, st, ws, (int)nch, pooled, W1, W2, hbuf, wts, beta, gW1,
                     gb1, gW2, gb2, N, MC, Hd, M, V, accumulate);
  return mmseg::check_launch("attn_gate_bwd");
}

}  // extern "C"
