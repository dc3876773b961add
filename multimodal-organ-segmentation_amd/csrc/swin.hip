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
__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_grad(float x) {
  return 0.5f * (1.f + erff(x * 0.70710678118654752f)) + x * 0.39894228040143268f * __expf(-0.5f * x * x);
}

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
// y = lrelu((a - ma) * ra + R), R = (b - mb) * rb | b | 0; stats [n][C]
template <typename T>
__global__ void res_apply_kernel(const T* __restrict__ a, int lda, const float* __restrict__ ma,
                                 const float* __restrict__ ra, const T* __restrict__ b, int ldb,
                                 const float* __restrict__ mb, const float* __restrict__ rb, T* __restrict__ y, int ldy,
                                 long long V, int C, float slope, long long total8) {
  const int c8n = C / 8;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total8;
       e += (long long)gridDim.x * blockDim.x) {
    const int c8 = (int)(e % c8n);
    const long long t = e / c8n;
    const int n = (int)(t / V);
    V8<T> va;
    va.load(a + t * lda + c8 * 8);
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c8 * 8 + j;
      o[j] = (va.get(j) - ma[n * C + c]) * ra[n * C + c];
    }
    if (b) {
      V8<T> vb;
      vb.load(b + t * ldb + c8 * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = c8 * 8 + j;
        o[j] += mb ? (vb.get(j) - mb[n * C + c]) * rb[n * C + c] : vb.get(j);
      }
    }
    V8<T> vy;
#pragma unroll
    for (int j = 0; j < 8; ++j) vy.set(j, o[j] > 0.f ? o[j] : o[j] * slope);
    vy.store(y + t * ldy + c8 * 8);
  }
}

// g = dy * (y > 0 ? 1 : slope)   (g may alias dy)
template <typename T>
__global__ void lrelu_bwd_kernel(const T* __restrict__ y, int ldy, const T* dy, int lddy, T* g, int ldg, int C,
                                 float slope, long long total8) {
  const int c8n = C / 8;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total8;
       e += (long long)gridDim.x * blockDim.x) {
    const int c8 = (int)(e % c8n);
    const long long t = e / c8n;
    V8<T> vy, vd;
    vy.load(y + t * ldy + c8 * 8);
    vd.load(dy + t * lddy + c8 * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) vd.set(j, vy.get(j) > 0.f ? vd.get(j) : vd.get(j) * slope);
    vd.store(g + t * ldg + c8 * 8);
  }
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

template <typename T>
int ln_fwd_t(const void* x, int ldx, void* y, int ldy, long long rows, int C, const float* gamma, const float* beta,
             float eps, float* mean, float* rstd, hipStream_t s) {
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
             const float* gamma, const float* mean, const float* rstd, int add, float* part, hipStream_t s) {
  const int nl = ln_nl(C), nb = ln_blocks(rows);
  auto X = (const T*)x;
  auto G = (const T*)dy;
  auto O = (T*)dx;
#define LNB(NL) MMSEG_LAUNCH((layernorm_bwd_kernel<T, NL>), dim3(nb), dim3(256), 0, s, X, ldx, G, lddy, O, lddx, \
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
  return nb * LN_WAVES * 2LL * C;
}

int mmseg_layernorm_bwd(const void* x, int ldx, const void* dy, int lddy, void* dx, int lddx, long long rows, int C,
                        const float* gamma, const float* mean, const float* rstd, int add_dx, float* dgamma,
                        float* dbeta, int accumulate, float* ws, int dtype, void* stream) {
  MMSEG_REQUIRE(C >= 1 && C <= 3072 && rows >= 1, "layernorm_bwd: 1 <= C <= 3072 (got %d)", C);
  MMSEG_REQUIRE(!(dgamma || dbeta) || ws != nullptr, "layernorm_bwd: parameter gradients need the workspace");
  hipStream_t s = (hipStream_t)stream;
  float* part = (dgamma || dbeta) ? ws : nullptr;
  const int r = dtype == MMSEG_BF16
                    ? ln_bwd_t<bf16_t>(x, ldx, dy, lddy, dx, lddx, rows, C, gamma, mean, rstd, add_dx, part, s)
                    : ln_bwd_t<float>(x, ldx, dy, lddy, dx, lddx, rows, C, gamma, mean, rstd, add_dx, part, s);
  if (r || !part) return r;
  const int nb = ln_blocks(rows) * (64 * ln_nl(C) <= 1024 ? 1 : LN_WAVES);
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
                    const float* rb, void* y, int ldy, int N, long long V, int C, float slope, int dtype,
                    void* stream) {
  MMSEG_REQUIRE(C % 8 == 0, "res_apply: C %% 8 == 0");
  MMSEG_REQUIRE((mb == nullptr) == (rb == nullptr), "res_apply: mb and rb together or neither");
  const long long total8 = (long long)N * V * (C / 8);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMSEG_BF16)
    MMSEG_LAUNCH(res_apply_kernel<bf16_t>, dim3(grid_of(total8)), dim3(256), 0, s, (const bf16_t*)a, lda, ma,
                       ra, (const bf16_t*)b, ldb, mb, rb, (bf16_t*)y, ldy, V, C, slope, total8);
  else
    MMSEG_LAUNCH(res_apply_kernel<float>, dim3(grid_of(total8)), dim3(256), 0, s, (const float*)a, lda, ma, ra,
                       (const float*)b, ldb, mb, rb, (float*)y, ldy, V, C, slope, total8);
  return mmseg::check_launch("res_apply");
}

int mmseg_lrelu_bwd(const void* y, int ldy, const void* dy, int lddy, void* g, int ldg, long long rows, int C,
                    float slope, int dtype, void* stream) {
  MMSEG_REQUIRE(C % 8 == 0, "lrelu_bwd: C %% 8 == 0");
  const long long total8 = rows * (C / 8);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMSEG_BF16)
    MMSEG_LAUNCH(lrelu_bwd_kernel<bf16_t>, dim3(grid_of(total8)), dim3(256), 0, s, (const bf16_t*)y, ldy,
                       (const bf16_t*)dy, lddy, (bf16_t*)g, ldg, C, slope, total8);
  else
    MMSEG_LAUNCH(lrelu_bwd_kernel<float>, dim3(grid_of(total8)), dim3(256), 0, s, (const float*)y, ldy,
                       (const float*)dy, lddy, (float*)g, ldg, C, slope, total8);
  return mmseg::check_launch("lrelu_bwd");
}

}  // extern "C"
