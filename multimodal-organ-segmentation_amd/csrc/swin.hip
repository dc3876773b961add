// SwinUNETR token / residual-block kernels (reference swin_unetr.py:80-96 builds
// MONAI 1.3 SwinUNETR; MONAI is absent, so the semantics follow its published
// architecture: oracle/swin_oracle.py restates it and the tests hold the
// kernels to that restatement).
//
// Token tensors are channels-last [rows][ld] (the engine's NDHWC), rows =
// (b, z, y, x) tokens.  Every reduction is fixed-order (deterministic).
//
//   layernorm_fwd / _bwd   nn.LayerNorm(C) (norm1 / norm2 / PatchMerging.norm,
//                          and proj_out's affine-free F.layer_norm); one wave
//                          per token row, fp32 math, per-row mean / rstd kept
//                          for the backward; weight / bias gradients as
//                          per-block partials + a fixed-order column sum
//   gelu_fwd / _bwd        nn.GELU() (exact erf) of MLPBlock
//   window_partition       F.pad + torch.roll(-shift) + window_partition
//   window_reverse         window_reverse + torch.roll(+shift) + crop (+ the
//                          residual add shortcut + attn of the block)
//   merge_gather / _bwd    legacy PatchMerging sub-grid concat (pad odd sides)
//   patchify               PatchEmbed Conv3d(k2, s2) operand: NCDHW fp32 ->
//                          [tokens][Cin*8] (a 1x1 GEMM then applies the weights)
//   add                    residual x + mlp(x)
//   res_apply / lrelu_bwd  UnetResBlock tail: lrelu(IN(a) [+ IN(b) | + b]) and
//                          the LeakyReLU mask of its backward
#include "mmseg_common.h"

#include <algorithm>
#include <type_traits>
#include <cstdlib>

namespace {

constexpr int LN_WAVES = 4;   // rows per block pass

template <typename T>
__device__ __forceinline__ float ld_f(const T* p) { return to_f<T>(*p); }

// ------------------------------------------------------------------ LayerNorm
template <typename T, int NL>
__global__ __launch_bounds__(256) void layernorm_fwd_kernel(const T* __restrict__ x, int ldx, T* __restrict__ y,
                                                            int ldy, long long rows, int C,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta, float eps,
                                                            float* __restrict__ mean_out,
                                                            float* __restrict__ rstd_out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (long long r = (long long)blockIdx.x * LN_WAVES + wave; r < rows; r += (long long)gridDim.x * LN_WAVES) {
    const T* xr = x + r * ldx;
    float v[NL];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int c = lane + 64 * i;
      v[i] = c < C ? ld_f(xr + c) : 0.f;
      s += v[i];
    }
    const float mean = wave_sum(s) / (float)C;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int c = lane + 64 * i;
      const float d = c < C ? v[i] - mean : 0.f;
      q += d * d;
    }
    const float rstd = rsqrtf(wave_sum(q) / (float)C + eps);
    T* yr = y + r * ldy;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int c = lane + 64 * i;
      if (c < C) {
        float o = (v[i] - mean) * rstd;
        if (gamma) o = o * gamma[c] + beta[c];
        yr[c] = from_f<T>(o);
      }
    }
    if (lane == 0 && mean_out) {
      mean_out[r] = mean;
      rstd_out[r] = rstd;
    }
  }
}

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)), g = dy * gamma; dx (+)= when add.  Per-block column
// partials of dy * xhat (dgamma) and dy (dbeta): part[blk][2][C].
template <typename T, int NL>
__global__ __launch_bounds__(256) void layernorm_bwd_kernel(const T* __restrict__ x, int ldx, const T* __restrict__ dy,
                                                            int lddy, T* __restrict__ dx, int lddx, long long rows,
                                                            int C, const float* __restrict__ gamma,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ rstd, int add,
                                                            float* __restrict__ part) {
  __shared__ float red[LN_WAVES][2][64 * NL > 1024 ? 1 : 64 * NL];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float pg[NL], pb[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) pg[i] = pb[i] = 0.f;
  for (long long r = (long long)blockIdx.x * LN_WAVES + wave; r < rows; r += (long long)gridDim.x * LN_WAVES) {
    const T* xr = x + r * ldx;
    const T* dr = dy + r * lddy;
    const float mu = mean[r], rs = rstd[r];
    float xh[NL], g[NL];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int c = lane + 64 * i;
      float d = 0.f, h = 0.f;
      if (c < C) {
        d = ld_f(dr + c);
        h = (ld_f(xr + c) - mu) * rs;
      }
      xh[i] = h;
      pg[i] += d * h;
      pb[i] += d;
      g[i] = (c < C && gamma) ? d * gamma[c] : d;
      sg += g[i];
      sgx += g[i] * h;
    }
    const float mg = wave_sum(sg) / (float)C, mgx = wave_sum(sgx) / (float)C;
    T* o = dx + r * lddx;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int c = lane + 64 * i;
      if (c < C) {
        float v = rs * (g[i] - mg - xh[i] * mgx);
        if (add) v += ld_f(o + c);
        o[c] = from_f<T>(v);
      }
    }
  }
  if (part == nullptr) return;
  if constexpr (64 * NL <= 1024) {
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      red[wave][0][lane + 64 * i] = pg[i];
      red[wave][1][lane + 64 * i] = pb[i];
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int w = 0; w < LN_WAVES; ++w) {
        a += red[w][0][c];
        b += red[w][1][c];
      }
      part[((long long)blockIdx.x * 2) * C + c] = a;
      part[((long long)blockIdx.x * 2 + 1) * C + c] = b;
    }
  } else {
    // wide rows: per-wave partials straight to global (part[blk*LN_WAVES + wave][2][C])
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int c = lane + 64 * i;
      if (c < C) {
        part[((long long)(blockIdx.x * LN_WAVES + wave) * 2) * C + c] = pg[i];
        part[((long long)(blockIdx.x * LN_WAVES + wave) * 2 + 1) * C + c] = pb[i];
      }
    }
  }
}

// ---------------------------------------------------- LayerNorm, row groups (r05)
// The kernels above give each token row a whole wave with one 2-byte element per lane: at the SwinUNETR widths
// (C = 48 at stage 0: 48 active lanes of 64, 96 B per row) a wave spends two dependent wave-wide reductions and
// two memory latencies on 96 bytes, and the launch ran at 0.75 (fwd) / 1.1 (bwd) TB/s (r05c c4 PMC).  Here a row
// belongs to G lanes (G = the power of two >= C / 8, <= 64), each holding V vectors of 8 channels (16-B loads),
// so a wave carries 64 / G rows; the row sums are xor-shuffle trees over the G lanes, and every lane keeps two
// rows in flight.  Same two-pass mean / variance in fp32 (not the same summation order as the wave-per-row form).
// The backward writes per-wave dgamma / dbeta partials part[(block * 4 + wave)][2][C] (ln_param_reduce sums them
// in a fixed order).
constexpr int LNG_LDS_C = 768;   // widest row whose per-block dgamma / dbeta partial is reduced in LDS

template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T, int G, int V>
__global__ __launch_bounds__(256) void layernorm_fwd_g_kernel(const T* __restrict__ x, int ldx, T* __restrict__ y,
                                                              int ldy, long long rows, int C,
                                                              const float* __restrict__ gamma,
                                                              const float* __restrict__ beta, float eps,
                                                              float* __restrict__ mean_out,
                                                              float* __restrict__ rstd_out) {
  constexpr int RPW = 64 / G, U = 2;                 // rows per wave, row iterations in flight per lane
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int gl = lane & (G - 1), gr = lane / G;
  float ga[V][8], be[V][8];
  bool cok[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const int c = (gl + G * v) * 8;
    cok[v] = c < C;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ga[v][j] = (gamma && cok[v]) ? gamma[c + j] : 1.f;
      be[v][j] = (beta && cok[v]) ? beta[c + j] : 0.f;
    }
  }
  const float invC = 1.f / (float)C;
  const long long step = (long long)gridDim.x * 4 * RPW;
  for (long long base = ((long long)blockIdx.x * 4 + wave) * RPW; base < rows; base += U * step) {
    V8<T> xv[U][V];
    long long r[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      r[u] = base + u * step + gr;
      ok[u] = r[u] < rows;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        if (ok[u] && cok[v]) xv[u][v].load(x + r[u] * ldx + (gl + G * v) * 8);
        else xv[u][v].zero();
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float s = 0.f;
#pragma unroll
      for (int v = 0; v < V; ++v)
#pragma unroll
        for (int j = 0; j < 8; ++j) s += xv[u][v].get(j);
      const float mean = group_sum<G>(s) * invC;
      float q = 0.f;
#pragma unroll
      for (int v = 0; v < V; ++v)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = cok[v] ? xv[u][v].get(j) - mean : 0.f;
          q += d * d;
        }
      const float rs = rsqrtf(group_sum<G>(q) * invC + eps);
      if (ok[u]) {
#pragma unroll
        for (int v = 0; v < V; ++v) {
          if (!cok[v]) continue;
          V8<T> o;
#pragma unroll
          for (int j = 0; j < 8; ++j) o.set(j, (xv[u][v].get(j) - mean) * rs * ga[v][j] + be[v][j]);
          o.store(y + r[u] * ldy + (gl + G * v) * 8);
        }
        if (gl == 0 && mean_out) {
          mean_out[r[u]] = mean;
          rstd_out[r[u]] = rs;
        }
      }
    }
  }
}

template <typename T, int G, int V>
__global__ __launch_bounds__(256) void layernorm_bwd_g_kernel(const T* __restrict__ x, int ldx,
                                                              const T* __restrict__ dy, int lddy, T* __restrict__ dx,
                                                              int lddx, long long rows, int C,
                                                              const float* __restrict__ gamma,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ rstd, int add,
                                                              float* __restrict__ part) {
  constexpr int RPW = 64 / G, U = 2;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int gl = lane & (G - 1), gr = lane / G;
  float ga[V][8], pg[V][8], pb[V][8];
  bool cok[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const int c = (gl + G * v) * 8;
    cok[v] = c < C;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ga[v][j] = (gamma && cok[v]) ? gamma[c + j] : 1.f;
      pg[v][j] = pb[v][j] = 0.f;
    }
  }
  const float invC = 1.f / (float)C;
  const long long step = (long long)gridDim.x * 4 * RPW;
  for (long long base = ((long long)blockIdx.x * 4 + wave) * RPW; base < rows; base += U * step) {
    V8<T> xv[U][V], dv[U][V];
    long long r[U];
    bool ok[U];
    float mu[U], rs[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      r[u] = base + u * step + gr;
      ok[u] = r[u] < rows;
      mu[u] = ok[u] ? mean[r[u]] : 0.f;
      rs[u] = ok[u] ? rstd[r[u]] : 0.f;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        if (ok[u] && cok[v]) {
          xv[u][v].load(x + r[u] * ldx + (gl + G * v) * 8);
          dv[u][v].load(dy + r[u] * lddy + (gl + G * v) * 8);
        } else {
          xv[u][v].zero();
          dv[u][v].zero();
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float sg = 0.f, sgx = 0.f;
#pragma unroll
      for (int v = 0; v < V; ++v)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = dv[u][v].get(j), h = (xv[u][v].get(j) - mu[u]) * rs[u];
          pg[v][j] += d * h;      // (padding rows / channels: d = 0)
          pb[v][j] += d;
          const float gg = d * ga[v][j];
          sg += gg;
          sgx += gg * h;
        }
      const float mg = group_sum<G>(sg) * invC, mgx = group_sum<G>(sgx) * invC;
      if (!ok[u]) continue;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        if (!cok[v]) continue;
        T* o = dx + r[u] * lddx + (gl + G * v) * 8;
        V8<T> prev, out;
        if (add) prev.load(o);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float h = (xv[u][v].get(j) - mu[u]) * rs[u];
          float w = rs[u] * (dv[u][v].get(j) * ga[v][j] - mg - h * mgx);
          if (add) w += prev.get(j);
          out.set(j, w);
        }
        out.store(o);
      }
    }
  }
  if (part == nullptr) return;
  // partials of the wave: the RPW row groups of the wave hold the same channels -- fixed xor tree over them
#pragma unroll
  for (int v = 0; v < V; ++v)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
      for (int o = G; o < 64; o <<= 1) {
        pg[v][j] += __shfl_xor(pg[v][j], o, 64);
        pb[v][j] += __shfl_xor(pb[v][j], o, 64);
      }
    }
  if constexpr (G * V * 8 <= LNG_LDS_C) {
    // C <= 768: the 4 waves' partials summed in LDS (wave order), one partial row pair per block
    __shared__ float red[4][2][LNG_LDS_C];
    if (gr == 0) {
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const int c = (gl + G * v) * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          red[wave][0][c + j] = pg[v][j];
          red[wave][1][c + j] = pb[v][j];
        }
      }
    }
    __syncthreads();
    float* pw = part + (long long)blockIdx.x * 2 * C;
    for (int e = threadIdx.x; e < 2 * C; e += 256) {
      const int k = e >= C, c = e - k * C;
      pw[e] = ((red[0][k][c] + red[1][k][c]) + red[2][k][c]) + red[3][k][c];
    }
  } else if (gr == 0) {
    float* pw = part + (long long)(blockIdx.x * 4 + wave) * 2 * C;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      if (!cok[v]) continue;
      const int c = (gl + G * v) * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        pw[c + j] = pg[v][j];
        pw[C + c + j] = pb[v][j];
      }
    }
  }
}

// out[c] (+)= sum_b part[b][k][C] over b, k = 0 (dgamma) / 1 (dbeta).  Block = 64 columns x 16 waves: wave w
// sums partial rows w, w+16, ... (8 loads in flight), then the 16 wave sums are added in wave order (fixed).
constexpr int LNR_WAVES = 16;
__global__ __launch_bounds__(1024) void ln_param_reduce_kernel(const float* __restrict__ part, int nb, int C,
                                                               float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                               int accumulate) {
  __shared__ float red[LNR_WAVES][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;           // column of [2][C]
  const bool ok = c < 2 * C;
  const int k = ok ? c / C : 0, cc = ok ? c - k * C : 0;
  float s = 0.f;
  if (ok) {
    const float* p = part + (long long)k * C + cc;
    const long long stride = 2LL * C;
    int b = wave;
    for (; b + 7 * LNR_WAVES < nb; b += 8 * LNR_WAVES) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = p[(long long)(b + j * LNR_WAVES) * stride];
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[j];
    }
    for (; b < nb; b += LNR_WAVES) s += p[(long long)b * stride];
  }
  red[wave][lane] = s;
  __syncthreads();
  if (wave != 0 || !ok) return;
  float t = 0.f;
#pragma unroll
  for (int w = 0; w < LNR_WAVES; ++w) t += red[w][lane];
  float* out = k == 0 ? dgamma : dbeta;
  if (out) out[cc] = accumulate ? out[cc] + t : t;
}

// ------------------------------------------------------------------ GELU
__device__ __forceinline__ float gelu_f(float x) { return mmseg_gelu(x); }
__device__ __forceinline__ float gelu_grad(float x) { return mmseg_gelu_grad(x); }

template <typename T>
__global__ void gelu_fwd_kernel(const T* __restrict__ h, T* __restrict__ y, long long n8) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    V8<T> a;
    a.load(h + i * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) a.set(j, gelu_f(a.get(j)));
    a.store(y + i * 8);
  }
}

template <typename T>
__global__ void gelu_bwd_kernel(const T* __restrict__ h, const T* __restrict__ dy, T* __restrict__ dh, long long n8) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    V8<T> a, d;
    a.load(h + i * 8);
    d.load(dy + i * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) d.set(j, d.get(j) * gelu_grad(a.get(j)));
    d.store(dh + i * 8);
  }
}

template <typename T>
__global__ void add_kernel(const T* __restrict__ a, const T* __restrict__ b, T* __restrict__ out, long long n8) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    V8<T> x, y;
    x.load(a + i * 8);
    y.load(b + i * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) x.set(j, x.get(j) + y.get(j));
    x.store(out + i * 8);
  }
}

// ------------------------------------------------------------ dropout
// nn.Dropout(p) of MONAI SwinUNETR's drop_rate sites (pos_drop, WindowAttention.proj_drop, MLPBlock
// drop1 / drop2).  Counter-based: the element with hash index h is kept iff the top 32 bits of
// splitmix64(seed + h * 0x9E3779B97F4A7C15) are >= thr = p * 2^32, and a kept element is scaled by
// 1 / (1 - p).  The backward applies the same call (same seed) to the gradient, so no mask is stored.
// h is the flat index of a [rows][C] channels-last buffer, or (ncdhw) the element's index in NCDHW order
// with rows = N * V (pos_drop acts on patch_embed's NCDHW output).
__device__ __forceinline__ unsigned int drop_hash(unsigned long long seed, unsigned long long h) {
  unsigned long long z = seed + h * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (unsigned int)(z >> 32);
}

template <typename T>
__global__ void dropout_kernel(const T* __restrict__ x, T* __restrict__ y, long long n8, int C, long long V,
                               int ncdhw, unsigned long long seed, unsigned int thr, float scale) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    V8<T> a;
    a.load(x + i * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const long long e = i * 8 + j;
      long long h = e;
      if (ncdhw) {
        const long long r = e / C, c = e - r * C, n = r / V, v = r - n * V;
        h = (n * C + c) * V + v;
      }
      a.set(j, drop_hash(seed, (unsigned long long)h) >= thr ? a.get(j) * scale : 0.f);
    }
    a.store(y + i * 8);
  }
}

// ------------------------------------------------------------ windows
struct WinArgs {
  int B, D, H, W, C;        // real grid and channels
  int w0, w1, w2;           // window
  int s0, s1, s2;           // shift (roll by -s before partition)
  int Dp, Hp, Wp;           // padded grid (multiples of the window)
  int ldx;                  // row stride of the grid tensor
};

// dst[(b*nW + win)*N + n][C] = padded-rolled grid at the window slot (0 in the padding)
template <typename T>
__global__ void window_partition_kernel(const T* __restrict__ src, WinArgs a, T* __restrict__ dst, long long total8) {
  const int c8n = a.C / 8;
  const int N = a.w0 * a.w1 * a.w2;
  const int nz = a.Dp / a.w0, ny = a.Hp / a.w1, nx = a.Wp / a.w2;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total8;
       e += (long long)gridDim.x * blockDim.x) {
    const int c8 = (int)(e % c8n);
    long long t = e / c8n;
    const int n = (int)(t % N);
    long long wi = t / N;
    const int wx = (int)(wi % nx); wi /= nx;
    const int wy = (int)(wi % ny); wi /= ny;
    const int wz = (int)(wi % nz);
    const int b = (int)(wi / nz);
    const int iz = n / (a.w1 * a.w2), iy = (n / a.w2) % a.w1, ix = n % a.w2;
    int z = wz * a.w0 + iz + a.s0, y = wy * a.w1 + iy + a.s1, x = wx * a.w2 + ix + a.s2;
    z -= z >= a.Dp ? a.Dp : 0;
    y -= y >= a.Hp ? a.Hp : 0;
    x -= x >= a.Wp ? a.Wp : 0;
    V8<T> v;
    if (z < a.D && y < a.H && x < a.W)
      v.load(src + (((long long)b * a.D + z) * a.H * a.W + (long long)y * a.W + x) * a.ldx + c8 * 8);
    else
      v.zero();
    v.store(dst + t * a.C + c8 * 8);
  }
}

// grid[b,z,y,x] = (add ? add_src[b,z,y,x] : 0) + win[slot of the rolled position], real tokens only
template <typename T>
__global__ void window_reverse_kernel(const T* __restrict__ win, WinArgs a, const T* __restrict__ add_src, int ld_add,
                                      T* __restrict__ dst, int ld_dst, long long total8) {
  const int c8n = a.C / 8;
  const int nz = a.Dp / a.w0, ny = a.Hp / a.w1, nx = a.Wp / a.w2;
  const int N = a.w0 * a.w1 * a.w2;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total8;
       e += (long long)gridDim.x * blockDim.x) {
    const int c8 = (int)(e % c8n);
    long long t = e / c8n;
    const int x = (int)(t % a.W);
    long long q = t / a.W;
    const int y = (int)(q % a.H);
    q /= a.H;
    const int z = (int)(q % a.D);
    const int b = (int)(q / a.D);
    int jz = z - a.s0, jy = y - a.s1, jx = x - a.s2;
    jz += jz < 0 ? a.Dp : 0;
    jy += jy < 0 ? a.Hp : 0;
    jx += jx < 0 ? a.Wp : 0;
    const long long wi = (((long long)b * nz + jz / a.w0) * ny + jy / a.w1) * nx + jx / a.w2;
    const int n = ((jz % a.w0) * a.w1 + jy % a.w1) * a.w2 + jx % a.w2;
    V8<T> v;
    v.load(win + (wi * N + n) * a.C + c8 * 8);
    if (add_src) {
      V8<T> r;
      r.load(add_src + t * ld_add + c8 * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) v.set(j, r.get(j) + v.get(j));
    }
    v.store(dst + t * ld_dst + c8 * 8);
  }
}

// ------------------------------------------------------- patch merging
// MONAI legacy PatchMerging sub-grid order (z, y, x parity per concat slot k)
__constant__ int kMergeOff[8][3] = {{0, 0, 0}, {1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {1, 0, 1}, {0, 1, 0}, {0, 0, 1},
                                    {1, 1, 1}};

template <typename T>
__global__ void merge_gather_kernel(const T* __restrict__ x, int ldx, int B, int D, int H, int W, int C,
                                    T* __restrict__ out, long long total8) {
  const int D2 = (D + 1) / 2, H2 = (H + 1) / 2, W2 = (W + 1) / 2;
  const int c8n = C / 8;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total8;
       e += (long long)gridDim.x * blockDim.x) {
    const int c8 = (int)(e % c8n);
    long long t = e / c8n;
    const int k = (int)(t % 8);
    t /= 8;
    const int x2 = (int)(t % W2);
    long long q = t / W2;
    const int y2 = (int)(q % H2);
    q /= H2;
    const int z2 = (int)(q % D2);
    const int b = (int)(q / D2);
    const int z = 2 * z2 + kMergeOff[k][0], y = 2 * y2 + kMergeOff[k][1], xx = 2 * x2 + kMergeOff[k][2];
    V8<T> v;
    if (z < D && y < H && xx < W)
      v.load(x + (((long long)b * D + z) * H * W + (long long)y * W + xx) * ldx + c8 * 8);
    else
      v.zero();
    v.store(out + (t * 8 + k) * C + c8 * 8);
  }
}

// dx[b,z,y,x][c] = sum over slots k whose parity is (z&1, y&1, x&1) of dout[b,z/2,y/2,x/2][k*C+c] (k ascending)
template <typename T>
__global__ void merge_scatter_kernel(const T* __restrict__ dout, int B, int D, int H, int W, int C,
                                     T* __restrict__ dx, int lddx, long long total8) {
  const int D2 = (D + 1) / 2, H2 = (H + 1) / 2, W2 = (W + 1) / 2;
  const int c8n = C / 8;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total8;
       e += (long long)gridDim.x * blockDim.x) {
    const int c8 = (int)(e % c8n);
    long long t = e / c8n;
    const int xx = (int)(t % W);
    long long q = t / W;
    const int y = (int)(q % H);
    q /= H;
    const int z = (int)(q % D);
    const int b = (int)(q / D);
    const long long t2 = (((long long)b * D2 + z / 2) * H2 + y / 2) * W2 + xx / 2;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (kMergeOff[k][0] == (z & 1) && kMergeOff[k][1] == (y & 1) && kMergeOff[k][2] == (xx & 1)) {
        V8<T> v;
        v.load(dout + (t2 * 8 + k) * C + c8 * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += v.get(j);
      }
    }
    V8<T> o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o.set(j, acc[j]);
    o.store(dx + t * lddx + c8 * 8);
  }
}

// -------------------------------------------------------------- patchify
// out[t][ci*8 + kz*4 + ky*2 + kx] = x[b][ci][2z+kz][2y+ky][2x+kx]; columns K..Kp-1 zero
template <typename T>
__global__ void patchify_kernel(const float* __restrict__ x, int B, int Cin, int D, int H, int W, int Kp,
                                T* __restrict__ out, long long total) {
  const int D2 = D / 2, H2 = H / 2, W2 = W / 2;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int col = (int)(e % Kp);
    const long long t = e / Kp;
    float v = 0.f;
    if (col < Cin * 8) {
      const int ci = col / 8, kz = (col >> 2) & 1, ky = (col >> 1) & 1, kx = col & 1;
      const int x2 = (int)(t % W2);
      long long q = t / W2;
      const int y2 = (int)(q % H2);
      q /= H2;
      const int z2 = (int)(q % D2);
      const int b = (int)(q / D2);
      v = x[((((long long)b * Cin + ci) * D + 2 * z2 + kz) * H + 2 * y2 + ky) * W + 2 * x2 + kx];
    }
    out[e] = from_f<T>(v);
  }
}

// ------------------------------------------------------ UnetResBlock tail
constexpr int RU = 4;   // rows in flight per thread
// Whole-row writes: a pass over C real channels of rows with pitch ld > C (SwinUNETR's 48 / 96 channels stored as 64
// / 128) also writes zeros into the row's padding [C, Cw) (npad = (Cw - C) / 8 <= C / 8 groups, one per thread of the
// row's first groups), so every 128-B line is written whole: a pass writing 96 B of each 128-B row ran at ~60 % of
// the whole-row rate (tools/diag_rows.py, r05k: res_apply 235 us at 48 / 64 vs 178 us at 64 / 64 real channels).
// The padding holds zeros anyway (zero-filled buffers whose pad columns nothing else writes).
template <typename T>
__device__ __forceinline__ void store_zero8(T* p) {
  V8<T> z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z.set(j, 0.f);
  z.store(p);
}
// Row-group layout: thread = (row lane tr, 8-channel group c8), rpb = 256 / (C / 8) rows per block pass, so the
// (row, channel) split is one 32-bit division per thread instead of two 64-bit divisions per 16-B access (which
// held these passes to ~2.7 TB/s at 128^3, r05c timer).
// y = lrelu((a - ma) * ra + R), R = (b - mb) * rb | b | 0; stats [n][C]; grid (row blocks, N)
template <typename T, bool ZP>
__global__ __launch_bounds__(256) void res_apply_kernel(const T* __restrict__ a, int lda, const float* __restrict__ ma,
                                                        const float* __restrict__ ra, const T* __restrict__ b, int ldb,
                                                        const float* __restrict__ mb, const float* __restrict__ rb,
                                                        T* __restrict__ y, int ldy, int V, int C, float slope,
                                                        int npad) {
  const int c8n = C >> 3, rpb = 256 / c8n;
  const int tr = threadIdx.x / c8n, c8 = threadIdx.x - tr * c8n;
  if (tr >= rpb) return;
  const int n = blockIdx.y, c0 = n * C + c8 * 8;
  float mua[8], rsa[8], mub[8], rsb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mua[j] = ma[c0 + j];
    rsa[j] = ra[c0 + j];
    mub[j] = mb ? mb[c0 + j] : 0.f;
    rsb[j] = mb ? rb[c0 + j] : 0.f;
  }
  const long long base = (long long)n * V;
  const int step = gridDim.x * rpb;
  // RU rows in flight per thread: all their loads issue before the first is used
  for (int v0 = blockIdx.x * rpb + tr; v0 < V; v0 += RU * step) {
    V8<T> va[RU], vb[RU];
#pragma unroll
    for (int u = 0; u < RU; ++u)
      if (v0 + u * step < V) {
        const long long t = base + v0 + u * step;
        va[u].load(a + t * lda + c8 * 8);
        if (b) vb[u].load(b + t * ldb + c8 * 8);
      }
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      if (v0 + u * step >= V) break;
      const long long t = base + v0 + u * step;
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (va[u].get(j) - mua[j]) * rsa[j];
      if (b) {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] += mb ? (vb[u].get(j) - mub[j]) * rsb[j] : vb[u].get(j);
      }
      V8<T> vy;
#pragma unroll
      for (int j = 0; j < 8; ++j) vy.set(j, o[j] > 0.f ? o[j] : o[j] * slope);
      vy.store(y + t * ldy + c8 * 8);
      if constexpr (ZP) {
        if (c8 < npad) store_zero8(y + t * ldy + C + c8 * 8);
      }
    }
  }
}

// g = dy * (y > 0 ? 1 : slope)   (g may alias dy); same row-group layout over rows rows
template <typename T, bool ZP>
__global__ __launch_bounds__(256) void lrelu_bwd_kernel(const T* __restrict__ y, int ldy, const T* dy, int lddy, T* g,
                                                        int ldg, int C, float slope, int rows, int npad) {
  const int c8n = C >> 3, rpb = 256 / c8n;
  const int tr = threadIdx.x / c8n, c8 = threadIdx.x - tr * c8n;
  if (tr >= rpb) return;
  const int step = gridDim.x * rpb;
  for (int r0 = blockIdx.x * rpb + tr; r0 < rows; r0 += RU * step) {
    V8<T> vy[RU], vd[RU];
#pragma unroll
    for (int u = 0; u < RU; ++u)
      if (r0 + u * step < rows) {
        const long long t = r0 + u * step;
        vy[u].load(y + t * ldy + c8 * 8);
        vd[u].load(dy + t * lddy + c8 * 8);
      }
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      if (r0 + u * step >= rows) break;
      const long long t = r0 + u * step;
#pragma unroll
      for (int j = 0; j < 8; ++j) vd[u].set(j, vy[u].get(j) > 0.f ? vd[u].get(j) : vd[u].get(j) * slope);
      vd[u].store(g + t * ldg + c8 * 8);
      if constexpr (ZP) {
        if (c8 < npad) store_zero8(g + t * ldg + C + c8 * 8);
      }
    }
  }
}

// row blocks of the row-group layout: enough for ~16 K blocks in all, at least RU rows per thread
int row_blocks(long long rows, int C, int nsplit) {
  const int rpb = 256 / (C / 8);
  const long long need = (rows + (long long)rpb * RU - 1) / ((long long)rpb * RU);
  const long long cap = std::max(1, 16384 / std::max(1, nsplit));
  return (int)std::max(1LL, std::min(need, cap));
}

int grid_of(long long total) {
  long long b = (total + 255) / 256;
  return (int)(b < 16384 ? (b < 1 ? 1 : b) : 16384);
}

int ln_nl(int C) {
  const int q = (C + 63) / 64;
  const int opts[] = {1, 2, 4, 8, 16, 24, 48};
  for (int o : opts)
    if (q <= o) return o;
  return 0;
}

int ln_blocks(long long rows) {
  long long b = (rows + LN_WAVES - 1) / LN_WAVES;
  return (int)(b < 1024 ? (b < 1 ? 1 : b) : 1024);
}

// (G, V) of the row-group LayerNorm kernels for C (0: not covered -> the wave-per-row kernels)
int ln_gv(int C, int ldx, int ldy, int* V) {
  if (C % 8 || ldx % 8 || ldy % 8) return 0;
  const int c8 = C / 8;
  int G = 8;
  while (G < c8 && G < 64) G *= 2;
  *V = (c8 + G - 1) / G;
  if (c8 < 4) return 0;
  return (*V == 1 || *V == 2 || *V == 3 || *V == 6) ? G : 0;
}

int ln_g_blocks(long long rows, int G) {
  const long long per = 4LL * (64 / G) * 2;   // rows per block per loop iteration (U = 2)
  long long b = (rows + per - 1) / per;
  return (int)(b < 1024 ? (b < 1 ? 1 : b) : 1024);
}

template <typename T>
int ln_fwd_t(const void* x, int ldx, void* y, int ldy, long long rows, int C, const float* gamma, const float* beta,
             float eps, float* mean, float* rstd, hipStream_t s) {
  int V = 0;
  const int G = ln_gv(C, ldx, ldy, &V);
  if (G) {
    const int nb = ln_g_blocks(rows, G);
    mmseg::note_kernel("layernorm_fwd_g_kernel");
#define LNG(GG, VV) MMSEG_LAUNCH((layernorm_fwd_g_kernel<T, GG, VV>), dim3(nb), dim3(256), 0, s, (const T*)x, ldx, \
                                 (T*)y, ldy, rows, C, gamma, beta, eps, mean, rstd)
    if (G == 8) LNG(8, 1);
    else if (G == 16) LNG(16, 1);
    else if (G == 32) LNG(32, 1);
    else if (V == 1) LNG(64, 1);
    else if (V == 2) LNG(64, 2);
    else if (V == 3) LNG(64, 3);
    else LNG(64, 6);
#undef LNG
    return mmseg::check_launch("layernorm_fwd_g");
  }
  const int nl = ln_nl(C), nb = ln_blocks(rows);
  auto X = (const T*)x;
  auto Y = (T*)y;
#define LNF(NL) MMSEG_LAUNCH((layernorm_fwd_kernel<T, NL>), dim3(nb), dim3(256), 0, s, X, ldx, Y, ldy, rows, C, \
                                   gamma, beta, eps, mean, rstd)
  switch (nl) {
    case 1: LNF(1); break;
    case 2: LNF(2); break;
    case 4: LNF(4); break;
    case 8: LNF(8); break;
    case 16: LNF(16); break;
    case 24: LNF(24); break;
    default: LNF(48); break;
  }
#undef LNF
  return mmseg::check_launch("layernorm_fwd");
}

template <typename T>
int ln_bwd_t(const void* x, int ldx, const void* dy, int lddy, void* dx, int lddx, long long rows, int C,
             const float* gamma, const float* mean, const float* rstd, int add, float* part, hipStream_t s,
             int* part_rows) {
  int V = 0;
  const int G = (lddy % 8 == 0) ? ln_gv(C, ldx, lddx, &V) : 0;
  if (G) {
    const int nb = ln_g_blocks(rows, G);
    *part_rows = G * V * 8 <= LNG_LDS_C ? nb : nb * 4;
    mmseg::note_kernel("layernorm_bwd_g_kernel");
#define LNGB(GG, VV) MMSEG_LAUNCH((layernorm_bwd_g_kernel<T, GG, VV>), dim3(nb), dim3(256), 0, s, (const T*)x, ldx, \
                                  (const T*)dy, lddy, (T*)dx, lddx, rows, C, gamma, mean, rstd, add, part)
    if (G == 8) LNGB(8, 1);
    else if (G == 16) LNGB(16, 1);
    else if (G == 32) LNGB(32, 1);
    else if (V == 1) LNGB(64, 1);
    else if (V == 2) LNGB(64, 2);
    else if (V == 3) LNGB(64, 3);
    else LNGB(64, 6);
#undef LNGB
    return mmseg::check_launch("layernorm_bwd_g");
  }
  const int nl = ln_nl(C), nb = ln_blocks(rows);
  *part_rows = nb * (64 * ln_nl(C) <= 1024 ? 1 : LN_WAVES);
  auto X = (const T*)x;
  auto Gd = (const T*)dy;
  auto O = (T*)dx;
#define LNB(NL) MMSEG_LAUNCH((layernorm_bwd_kernel<T, NL>), dim3(nb), dim3(256), 0, s, X, ldx, Gd, lddy, O, lddx, \
                                   rows, C, gamma, mean, rstd, add, part)
  switch (nl) {
    case 1: LNB(1); break;
    case 2: LNB(2); break;
    case 4: LNB(4); break;
    case 8: LNB(8); break;
    case 16: LNB(16); break;
    case 24: LNB(24); break;
    default: LNB(48); break;
  }
#undef LNB
  return mmseg::check_launch("layernorm_bwd");
}

}  // namespace

extern "C" {

int mmseg_layernorm_fwd(const void* x, int ldx, void* y, int ldy, long long rows, int C, const float* gamma,
                        const float* beta, float eps, float* mean, float* rstd, int dtype, void* stream) {
  MMSEG_REQUIRE(C >= 1 && C <= 3072 && rows >= 1, "layernorm: 1 <= C <= 3072 (got %d), rows >= 1", C);
  MMSEG_REQUIRE((gamma == nullptr) == (beta == nullptr), "layernorm: gamma and beta together or neither");
  MMSEG_REQUIRE((mean == nullptr) == (rstd == nullptr), "layernorm: mean and rstd together or neither");
  hipStream_t s = (hipStream_t)stream;
  return dtype == MMSEG_BF16 ? ln_fwd_t<bf16_t>(x, ldx, y, ldy, rows, C, gamma, beta, eps, mean, rstd, s)
                             : ln_fwd_t<float>(x, ldx, y, ldy, rows, C, gamma, beta, eps, mean, rstd, s);
}

long long mmseg_layernorm_bwd_ws_floats(long long rows, int C) {
  const long long nb = ln_blocks(rows);
  // (the row-group kernels: at most 1,024 blocks x 4 per-wave partials)
  return std::max<long long>(nb * LN_WAVES, 1024LL * 4) * 2LL * C;
}

int mmseg_layernorm_bwd(const void* x, int ldx, const void* dy, int lddy, void* dx, int lddx, long long rows, int C,
                        const float* gamma, const float* mean, const float* rstd, int add_dx, float* dgamma,
                        float* dbeta, int accumulate, float* ws, int dtype, void* stream) {
  MMSEG_REQUIRE(C >= 1 && C <= 3072 && rows >= 1, "layernorm_bwd: 1 <= C <= 3072 (got %d)", C);
  MMSEG_REQUIRE(!(dgamma || dbeta) || ws != nullptr, "layernorm_bwd: parameter gradients need the workspace");
  hipStream_t s = (hipStream_t)stream;
  float* part = (dgamma || dbeta) ? ws : nullptr;
  int nb = 0;
  const int r = dtype == MMSEG_BF16
                    ? ln_bwd_t<bf16_t>(x, ldx, dy, lddy, dx, lddx, rows, C, gamma, mean, rstd, add_dx, part, s, &nb)
                    : ln_bwd_t<float>(x, ldx, dy, lddy, dx, lddx, rows, C, gamma, mean, rstd, add_dx, part, s, &nb);
  if (r || !part) return r;
  MMSEG_LAUNCH(ln_param_reduce_kernel, dim3(ceil_div(2LL * C, 64)), dim3(64 * LNR_WAVES), 0, s, part, nb, C,
                     dgamma, dbeta, accumulate);
  return mmseg::check_launch("ln_param_reduce");
}

int mmseg_gelu_fwd(const void* h, void* y, long long n, int dtype, void* stream) {
  MMSEG_REQUIRE(n % 8 == 0, "gelu: n %% 8 == 0");
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMSEG_BF16)
    MMSEG_LAUNCH(gelu_fwd_kernel<bf16_t>, dim3(grid_of(n / 8)), dim3(256), 0, s, (const bf16_t*)h, (bf16_t*)y,
                       n / 8);
  else
    MMSEG_LAUNCH(gelu_fwd_kernel<float>, dim3(grid_of(n / 8)), dim3(256), 0, s, (const float*)h, (float*)y,
                       n / 8);
  return mmseg::check_launch("gelu_fwd");
}

int mmseg_gelu_bwd(const void* h, const void* dy, void* dh, long long n, int dtype, void* stream) {
  MMSEG_REQUIRE(n % 8 == 0, "gelu_bwd: n %% 8 == 0");
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMSEG_BF16)
    MMSEG_LAUNCH(gelu_bwd_kernel<bf16_t>, dim3(grid_of(n / 8)), dim3(256), 0, s, (const bf16_t*)h,
                       (const bf16_t*)dy, (bf16_t*)dh, n / 8);
  else
    MMSEG_LAUNCH(gelu_bwd_kernel<float>, dim3(grid_of(n / 8)), dim3(256), 0, s, (const float*)h,
                       (const float*)dy, (float*)dh, n / 8);
  return mmseg::check_launch("gelu_bwd");
}

int mmseg_dropout(const void* x, void* y, long long rows, int C, long long V, int ncdhw, float p, long long seed,
                  int dtype, void* stream) {
  MMSEG_REQUIRE(rows * C % 8 == 0 && C > 0 && p >= 0.f && p < 1.f && (!ncdhw || (V > 0 && rows % V == 0)),
                "dropout: rows*C %% 8 == 0, 0 <= p < 1, rows a multiple of V");
  hipStream_t s = (hipStream_t)stream;
  const long long n8 = rows * C / 8;
  const double t = (double)p * 4294967296.0;
  const unsigned int thr = t >= 4294967295.0 ? 0xffffffffu : (unsigned int)t;
  const float scale = (float)(1.0 / (1.0 - (double)p));
  if (dtype == MMSEG_BF16)
    MMSEG_LAUNCH(dropout_kernel<bf16_t>, dim3(grid_of(n8)), dim3(256), 0, s, (const bf16_t*)x, (bf16_t*)y, n8,
                       C, V, ncdhw, (unsigned long long)seed, thr, scale);
  else
    MMSEG_LAUNCH(dropout_kernel<float>, dim3(grid_of(n8)), dim3(256), 0, s, (const float*)x, (float*)y, n8, C,
                       V, ncdhw, (unsigned long long)seed, thr, scale);
  return mmseg::check_launch("dropout");
}

int mmseg_add(const void* a, const void* b, void* out, long long n, int dtype, void* stream) {
  MMSEG_REQUIRE(n % 8 == 0, "add: n %% 8 == 0");
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMSEG_BF16)
    MMSEG_LAUNCH(add_kernel<bf16_t>, dim3(grid_of(n / 8)), dim3(256), 0, s, (const bf16_t*)a, (const bf16_t*)b,
                       (bf16_t*)out, n / 8);
  else
    MMSEG_LAUNCH(add_kernel<float>, dim3(grid_of(n / 8)), dim3(256), 0, s, (const float*)a, (const float*)b,
                       (float*)out, n / 8);
  return mmseg::check_launch("add");
}

static int win_check(const WinArgs& a) {
  MMSEG_REQUIRE(a.C % 8 == 0 && a.w0 > 0 && a.w1 > 0 && a.w2 > 0 && a.Dp % a.w0 == 0 && a.Hp % a.w1 == 0 &&
                    a.Wp % a.w2 == 0 && a.Dp >= a.D && a.Hp >= a.H && a.Wp >= a.W && a.s0 >= 0 && a.s0 < a.Dp &&
                    a.s1 >= 0 && a.s1 < a.Hp && a.s2 >= 0 && a.s2 < a.Wp,
                "window: C%%8, padded grid a multiple of the window, 0 <= shift < padded side");
  return 0;
}

int mmseg_window_partition(const void* src, int ldx, int B, int D, int H, int W, int C, int w0, int w1, int w2,
                           int s0, int s1, int s2, int Dp, int Hp, int Wp, void* dst, int dtype, void* stream) {
  WinArgs a{B, D, H, W, C, w0, w1, w2, s0, s1, s2, Dp, Hp, Wp, ldx};
  if (win_check(a)) return 1;
  const long long total8 = (long long)B * Dp * Hp * Wp * (C / 8);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMSEG_BF16)
    MMSEG_LAUNCH(window_partition_kernel<bf16_t>, dim3(grid_of(total8)), dim3(256), 0, s, (const bf16_t*)src, a,
                       (bf16_t*)dst, total8);
  else
    MMSEG_LAUNCH(window_partition_kernel<float>, dim3(grid_of(total8)), dim3(256), 0, s, (const float*)src, a,
                       (float*)dst, total8);
  return mmseg::check_launch("window_partition");
}

int mmseg_window_reverse(const void* win, int B, int D, int H, int W, int C, int w0, int w1, int w2, int s0, int s1,
                         int s2, int Dp, int Hp, int Wp, const void* add_src, int ld_add, void* dst, int ld_dst,
                         int dtype, void* stream) {
  WinArgs a{B, D, H, W, C, w0, w1, w2, s0, s1, s2, Dp, Hp, Wp, 0};
  if (win_check(a)) return 1;
  const long long total8 = (long long)B * D * H * W * (C / 8);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMSEG_BF16)
    MMSEG_LAUNCH(window_reverse_kernel<bf16_t>, dim3(grid_of(total8)), dim3(256), 0, s, (const bf16_t*)win, a,
                       (const bf16_t*)add_src, ld_add, (bf16_t*)dst, ld_dst, total8);
  else
    MMSEG_LAUNCH(window_reverse_kernel<float>, dim3(grid_of(total8)), dim3(256), 0, s, (const float*)win, a,
                       (const float*)add_src, ld_add, (float*)dst, ld_dst, total8);
  return mmseg::check_launch("window_reverse");
}

int mmseg_merge_gather(const void* x, int ldx, int B, int D, int H, int W, int C, void* out, int dtype, void* stream) {
  MMSEG_REQUIRE(C % 8 == 0, "merge_gather: C %% 8 == 0");
  const long long total8 = (long long)B * ((D + 1) / 2) * ((H + 1) / 2) * ((W + 1) / 2) * 8 * (C / 8);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMSEG_BF16)
    MMSEG_LAUNCH(merge_gather_kernel<bf16_t>, dim3(grid_of(total8)), dim3(256), 0, s, (const bf16_t*)x, ldx, B,
                       D, H, W, C, (bf16_t*)out, total8);
  else
    MMSEG_LAUNCH(merge_gather_kernel<float>, dim3(grid_of(total8)), dim3(256), 0, s, (const float*)x, ldx, B, D,
                       H, W, C, (float*)out, total8);
  return mmseg::check_launch("merge_gather");
}

int mmseg_merge_scatter(const void* dout, int B, int D, int H, int W, int C, void* dx, int lddx, int dtype,
                        void* stream) {
  MMSEG_REQUIRE(C % 8 == 0, "merge_scatter: C %% 8 == 0");
  const long long total8 = (long long)B * D * H * W * (C / 8);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMSEG_BF16)
    MMSEG_LAUNCH(merge_scatter_kernel<bf16_t>, dim3(grid_of(total8)), dim3(256), 0, s, (const bf16_t*)dout, B,
                       D, H, W, C, (bf16_t*)dx, lddx, total8);
  else
    MMSEG_LAUNCH(merge_scatter_kernel<float>, dim3(grid_of(total8)), dim3(256), 0, s, (const float*)dout, B, D,
                       H, W, C, (float*)dx, lddx, total8);
  return mmseg::check_launch("merge_scatter");
}

int mmseg_patchify(const float* x, int B, int Cin, int D, int H, int W, int Kp, void* out, int dtype, void* stream) {
  MMSEG_REQUIRE(D % 2 == 0 && H % 2 == 0 && W % 2 == 0 && Kp >= Cin * 8 && Kp % 8 == 0,
                "patchify: even sides and Kp >= 8*Cin, Kp %% 8 == 0");
  const long long total = (long long)B * (D / 2) * (H / 2) * (W / 2) * Kp;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMSEG_BF16)
    MMSEG_LAUNCH(patchify_kernel<bf16_t>, dim3(grid_of(total)), dim3(256), 0, s, x, B, Cin, D, H, W, Kp,
                       (bf16_t*)out, total);
  else
    MMSEG_LAUNCH(patchify_kernel<float>, dim3(grid_of(total)), dim3(256), 0, s, x, B, Cin, D, H, W, Kp,
                       (float*)out, total);
  return mmseg::check_launch("patchify");
}

int mmseg_res_apply(const void* a, int lda, const float* ma, const float* ra, const void* b, int ldb, const float* mb,
                    const float* rb, void* y, int ldy, int N, long long V, int C, int Cw, float slope, int dtype,
                    void* stream) {
  MMSEG_REQUIRE(C % 8 == 0 && C <= 2048, "res_apply: C %% 8 == 0 and C <= 2048");
  MMSEG_REQUIRE(Cw % 8 == 0 && Cw >= C && Cw <= 2 * C && Cw <= ldy, "res_apply: C <= Cw <= min(2 C, ldy), Cw %% 8 == 0");
  MMSEG_REQUIRE((mb == nullptr) == (rb == nullptr), "res_apply: mb and rb together or neither");
  MMSEG_REQUIRE(V < (1LL << 31), "res_apply: V must fit int32");
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(row_blocks(V, C, N), N);
  auto run = [&](auto tag, auto zp) {
    using T = decltype(tag);
    MMSEG_LAUNCH((res_apply_kernel<T, decltype(zp)::value>), grid, dim3(256), 0, s, (const T*)a, lda, ma, ra,
                 (const T*)b, ldb, mb, rb, (T*)y, ldy, (int)V, C, slope, (Cw - C) / 8);
  };
  if (dtype == MMSEG_BF16) {
    if (Cw > C) run(bf16_t{}, std::true_type{});
    else run(bf16_t{}, std::false_type{});
  } else {
    if (Cw > C) run(float{}, std::true_type{});
    else run(float{}, std::false_type{});
  }
  return mmseg::check_launch("res_apply");
}

int mmseg_lrelu_bwd(const void* y, int ldy, const void* dy, int lddy, void* g, int ldg, long long rows, int C, int Cw,
                    float slope, int dtype, void* stream) {
  MMSEG_REQUIRE(C % 8 == 0 && C <= 2048, "lrelu_bwd: C %% 8 == 0 and C <= 2048");
  MMSEG_REQUIRE(Cw % 8 == 0 && Cw >= C && Cw <= 2 * C && Cw <= ldg, "lrelu_bwd: C <= Cw <= min(2 C, ldg), Cw %% 8 == 0");
  MMSEG_REQUIRE(rows < (1LL << 31), "lrelu_bwd: rows must fit int32");
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(row_blocks(rows, C, 1));
  auto run = [&](auto tag, auto zp) {
    using T = decltype(tag);
    MMSEG_LAUNCH((lrelu_bwd_kernel<T, decltype(zp)::value>), grid, dim3(256), 0, s, (const T*)y, ldy, (const T*)dy,
                 lddy, (T*)g, ldg, C, slope, (int)rows, (Cw - C) / 8);
  };
  if (dtype == MMSEG_BF16) {
    if (Cw > C) run(bf16_t{}, std::true_type{});
    else run(bf16_t{}, std::false_type{});
  } else {
    if (Cw > C) run(float{}, std::true_type{});
    else run(float{}, std::false_type{});
  }
  return mmseg::check_launch("lrelu_bwd");
}

}  // extern "C"
