// Segmentation head, losses, metric and optimizer kernels.
//
//   head:   Dropout3d (per-(n,c) scale) + 1x1 Conv3d out_conv
//           (reference unet.py:162-163,195-196; dual_encoder.py:83-84,157-158)
//           NDHWC features -> NCDHW fp32 logits (the reference's output layout)
//   loss:   softmax over C + one-hot + per-(b,c) Dice / Tversky sums + CE in one
//           pass; fixed-order finalize; a second pass writes dlogits.
//           DiceLoss losses.py:39-80, DiceCELoss 216-228 (nn.CrossEntropyLoss
//           with optional class weights), TverskyLoss 160-185.
//   metric: argmax over C + per-class integer intersection / union counts
//           (DiceMetric.update, metrics.py:42-67) — integer, exact.
//   optim:  AdamW in torch's single-tensor op order (torch.optim.AdamW, as
//           configured by trainer.py:115-117), over flat parameter buffers.
//   input:  NCDHW fp32 volume -> NDHWC (8-channel padded) engine layout.
#include "mmseg_common.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>

namespace {

constexpr int CMAX = 16;

// -------------------------------------------------------------- input pack
template <typename T>
__global__ void pack_input_kernel(const float* __restrict__ x, int Ctot, int c0, int cnt, long long V, int N,
                                  T* __restrict__ out) {
  const long long total = (long long)N * V;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long n = i / V, v = i - n * V;
    V8<T> o;
    o.zero();
    for (int c = 0; c < cnt; ++c) o.set(c, x[(n * Ctot + c0 + c) * V + v]);
    o.store(out + i * 8);
  }
}

// compact variant for the stem: out[(n*V + v)*cnt + c], no channel padding
template <typename T>
__global__ void pack_input_compact_kernel(const float* __restrict__ x, int Ctot, int c0, int cnt, long long V, int N,
                                          T* __restrict__ out) {
  const long long total = (long long)N * V;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long n = i / V, v = i - n * V;
    for (int c = 0; c < cnt; ++c) out[i * cnt + c] = from_f<T>(x[(n * Ctot + c0 + c) * V + v]);
  }
}

// ----------------------------------------------------------------- head
// logits[n][c][v] = b[c] + sum_ci W[c][ci] * s[n][ci] * x[n,v,ci]
template <typename T>
__global__ void head_fwd_kernel(const T* __restrict__ x, int ldx, int Cin, const float* __restrict__ Wt,
                                const float* __restrict__ bias, const float* __restrict__ dscale, int C, long long V,
                                int N, float* __restrict__ logits) {
  extern __shared__ float sw[];  // C*Cin
  for (int i = threadIdx.x; i < C * Cin; i += blockDim.x) sw[i] = Wt[i];
  __syncthreads();
  const long long total = (long long)N * V;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long n = i / V, v = i - n * V;
    float acc[CMAX];
#pragma unroll
    for (int c = 0; c < CMAX; ++c) acc[c] = c < C ? bias[c] : 0.f;
    for (int cg = 0; cg < Cin / 8; ++cg) {
      V8<T> a;
      a.load(x + i * ldx + cg * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float xv = a.get(j);
        if (dscale) xv *= dscale[n * Cin + cg * 8 + j];
#pragma unroll
        for (int c = 0; c < CMAX; ++c)
          if (c < C) acc[c] = fmaf(sw[c * Cin + cg * 8 + j], xv, acc[c]);
      }
    }
#pragma unroll
    for (int c = 0; c < CMAX; ++c)
      if (c < C) logits[(n * C + c) * V + v] = acc[c];
  }
}

// Same head with the channel-group count CG = Cin / 8 known at compile time and
// U = 4 voxels per thread (i, i + S, i + 2S, i + 3S with S the grid's thread
// count): all U * CG 16-B feature loads are issued before any FMA, and one
// grid of total / (256 U) blocks covers the volume once.  The one-voxel form
// (one block per 256 voxels, each waiting on its weight preload and then on
// 64 B of loads per thread) ran at ~2.2 TB/s.
template <typename T, int CG, int CC>
__global__ __launch_bounds__(256) void head_fwd_u_kernel(const T* __restrict__ x, int ldx,
                                                         const float* __restrict__ Wt, const float* __restrict__ bias,
                                                         const float* __restrict__ dscale, long long V, int N,
                                                         float* __restrict__ logits) {
  constexpr int Cin = CG * 8, U = 4;
  __shared__ float sw[CC * Cin];
  for (int i = threadIdx.x; i < CC * Cin; i += blockDim.x) sw[i] = Wt[i];
  const long long total = (long long)N * V;
  const long long S = (long long)gridDim.x * blockDim.x;
  const long long i0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  V8<T> a[U][CG];
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (i0 + u * S < total)
#pragma unroll
      for (int cg = 0; cg < CG; ++cg) a[u][cg].load(x + (i0 + u * S) * ldx + cg * 8);
  __syncthreads();
  float acc[U][CC];
#pragma unroll
  for (int c = 0; c < CC; ++c) {
    const float b = bias[c];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u][c] = b;
  }
  // weights outer (read once from LDS per (ci, c)), the U voxels inner
#pragma unroll
  for (int cg = 0; cg < CG; ++cg)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float xv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        xv[u] = a[u][cg].get(j);
        if (dscale && i0 + u * S < total) xv[u] *= dscale[((i0 + u * S) / V) * Cin + cg * 8 + j];
      }
#pragma unroll
      for (int c = 0; c < CC; ++c) {
        const float w = sw[c * Cin + cg * 8 + j];
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u][c] = fmaf(w, xv[u], acc[u][c]);
      }
    }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long i = i0 + u * S;
    if (i >= total) break;
    const long long n = i / V, v = i - n * V;
#pragma unroll
    for (int c = 0; c < CC; ++c) logits[(n * CC + c) * V + v] = acc[u][c];
  }
}

// Tile-staged head for padded feature rows (SwinUNETR: 48 channels at pitch 64).  head_fwd_u gives each lane one
// voxel, so a wave's 16-B loads touch 64 rows 128 B apart (225 us at 128^3, ~1.4 TB/s, r05s).  Here a block stages
// HT_V consecutive voxels' CG 16-B groups with lanes on consecutive groups (each row's 96 B read by neighbouring
// lanes), converts them to fp32 in LDS, and then thread (voxel v = tid % HT_V, class slice) takes its classes'
// dot products from LDS: the logit stores of a class are consecutive voxels.  Same per-logit fma order as
// head_fwd_u (bias, then channels 0..Cin-1), so the logits are bitwise head_fwd_u's.
constexpr int HT_V = 128;
template <typename T, int CG, int CC>
__global__ __launch_bounds__(256) void head_fwd_t_kernel(const T* __restrict__ x, int ldx,
                                                         const float* __restrict__ Wt, const float* __restrict__ bias,
                                                         long long V, int N, float* __restrict__ logits) {
  constexpr int Cin = CG * 8, XP = Cin + 1;                  // fp32 row pitch (odd: conflict-free column reads)
  constexpr int CS = (CC + 1) / 2;                           // classes per thread (two class slices)
  __shared__ float sw[CC * Cin];
  __shared__ float xs[HT_V * XP];
  for (int i = threadIdx.x; i < CC * Cin; i += blockDim.x) sw[i] = Wt[i];
  const long long total = (long long)N * V;
  const int v = threadIdx.x % HT_V, half = threadIdx.x / HT_V;
  for (long long t0 = (long long)blockIdx.x * HT_V; t0 < total; t0 += (long long)gridDim.x * HT_V) {
    __syncthreads();   // the previous tile's reads are done (and, first time round, sw is written)
#pragma unroll
    for (int k = 0; k < (HT_V * CG + 255) / 256; ++k) {
      const int e = threadIdx.x + 256 * k;
      if (e < HT_V * CG) {
        const int r = e / CG, cg = e - r * CG;
        V8<T> a;
        if (t0 + r < total) a.load(x + (t0 + r) * ldx + cg * 8);
        else a.zero();
#pragma unroll
        for (int j = 0; j < 8; ++j) xs[r * XP + cg * 8 + j] = a.get(j);
      }
    }
    __syncthreads();
    const long long i = t0 + v;
    if (i < total) {
      const long long n = i / V, vv = i - n * V;
#pragma unroll
      for (int cc = 0; cc < CS; ++cc) {
        const int c = half * CS + cc;
        if (c < CC) {
          float acc = bias[c];
#pragma unroll 8
          for (int ci = 0; ci < Cin; ++ci) acc = fmaf(sw[c * Cin + ci], xs[v * XP + ci], acc);
          logits[(n * CC + c) * V + vv] = acc;
        }
      }
    }
  }
}

// dx[n,v,ci] = s[n][ci] * sum_c dlog[n][c][v] * W[c][ci]
template <typename T>
__global__ void head_dgrad_kernel(const float* __restrict__ dlog, const float* __restrict__ Wt,
                                  const float* __restrict__ dscale, int C, int Cin, long long V, int N,
                                  T* __restrict__ dx, int lddx) {
  extern __shared__ float sw[];
  for (int i = threadIdx.x; i < C * Cin; i += blockDim.x) sw[i] = Wt[i];
  __syncthreads();
  const long long total = (long long)N * V;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long n = i / V, v = i - n * V;
    float d[CMAX];
#pragma unroll
    for (int c = 0; c < CMAX; ++c) d[c] = c < C ? dlog[(n * C + c) * V + v] : 0.f;
    for (int cg = 0; cg < Cin / 8; ++cg) {
      V8<T> o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int ci = cg * 8 + j;
        float a = 0.f;
#pragma unroll
        for (int c = 0; c < CMAX; ++c)
          if (c < C) a = fmaf(d[c], sw[c * Cin + ci], a);
        if (dscale) a *= dscale[n * Cin + ci];
        o.set(j, a);
      }
      o.store(dx + i * lddx + cg * 8);
    }
  }
}


// Head data gradient, one lane per (voxel, 8-channel group): a wave stores consecutive voxels' groups (64 16-B
// lanes over ~64 B .. 1 KB of contiguous rows) whatever Cin / 8 is -- the quad-per-voxel form (lane q of 4 took the
// groups q, q + 4, ...) left SwinUNETR's 6 groups at 2 / 2 / 1 / 1 per quad (165 us at 128^3, 1.5 TB/s, r06y).
// The grid stride is a whole number of voxels (the last Cin/8 - 1 threads of the grid idle), so a lane keeps its
// group -- its 8 x C weights in registers -- and walks voxels without dividing.  Same per-channel fma order
// (classes 0..C-1 from 0, then the Dropout3d scale), so bitwise the quad form's dx.
template <typename T, int CM>   // CM >= C: classes held per lane (8 or CMAX)
__global__ __launch_bounds__(256) void head_dgrad_g_kernel(const float* __restrict__ dlog,
                                                           const float* __restrict__ Wt,
                                                           const float* __restrict__ dscale, int C, int Cin,
                                                           long long V, int N, T* __restrict__ dx, int lddx,
                                                           int Z8) {
  // Z8 >= Cin / 8 groups per row are written: the groups past Cin get zeros (whole 128-B rows of a view that owns
  // its padding, Act.wcols: a row's partial last line would cost the memory a read-modify-write)
  const int C8 = Cin >> 3;
  const long long G = (long long)gridDim.x * blockDim.x, gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long vstep = G / Z8;   // voxels per grid stride
  if (gid >= vstep * Z8) return;
  const int cg = (int)(gid % Z8);
  const bool real = cg < C8;
  float w[8][CM];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int c = 0; c < CM; ++c) w[j][c] = real && c < C ? Wt[c * Cin + cg * 8 + j] : 0.f;
  const long long total = (long long)N * V;
  long long i = gid / Z8;
  long long n = i / V, v = i - n * V;
  const long long nstep = vstep / V, vrem = vstep - nstep * V;
  // U voxels per round, all their dlogits loads issued before the first fma (one round trip per round)
  constexpr int U = 4;
  for (; i < total; i += U * vstep) {
    float d[U][CM];
    long long nu[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      nu[u] = n;
      const bool ok = real && i + u * vstep < total;
#pragma unroll
      for (int c = 0; c < CM; ++c) d[u][c] = ok && c < C ? dlog[(n * C + c) * V + v] : 0.f;
      n += nstep;
      v += vrem;
      if (v >= V) {
        v -= V;
        ++n;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (i + u * vstep >= total) break;
      V8<T> o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float a = 0.f;
#pragma unroll
        for (int c = 0; c < CM; ++c)
          if (c < C) a = fmaf(d[u][c], w[j][c], a);
        if (dscale && real) a *= dscale[nu[u] * Cin + cg * 8 + j];
        o.set(j, a);
      }
      o.store(dx + (i + u * vstep) * lddx + cg * 8);
    }
  }
}

// partial dW[c][ci] and db[c] per voxel chunk (block), fixed order.
// thread = (voxel lane, 8-channel group): vectorised x loads, 8x8 register tile per class chunk.
template <typename T>
__global__ __launch_bounds__(256) void head_wgrad_partial(const T* __restrict__ x, int ldx, const float* __restrict__ dlog,
                                   const float* __restrict__ dscale, int C, int Cin, long long V, int N,
                                   long long vpc, float* __restrict__ part) {
  __shared__ float red[256 * 8 + 4];
  const int C8 = Cin >> 3;
  // channel groups padded to a power of two (<= 32: the shuffle-tree reduction; SwinUNETR's 6 groups take 8 lanes,
  // 2 idle) -- the serial LDS sweep over 256 / C8 voxel lanes per class cost ~10 us per block at C8 = 6 (r06y)
  int C8p = 1;
  while (C8p < C8) C8p <<= 1;
  if (C8p > 32) C8p = C8;
  const int lanes_v = 256 / C8p;
  const int tid = threadIdx.x;
  const int cg = tid % C8p, vl = tid / C8p;
  const long long total = (long long)N * V;
  const long long e0 = (long long)blockIdx.x * vpc;
  long long e1 = e0 + vpc;
  if (e1 > total) e1 = total;
  const int npairs = C * Cin + C;
  for (int c0 = 0; c0 < C; c0 += 8) {
    float acc[8][8], bacc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      bacc[k] = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[k][j] = 0.f;
    }
    if (vl < lanes_v && cg < C8) {
      // U voxels per step: their feature and dlogits loads are issued before any FMA
      constexpr int U = 2;
      for (long long eb = e0 + vl; eb < e1; eb += U * lanes_v) {
        V8<T> a[U];
        float dd[U][8];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const long long e = eb + u * lanes_v;
          if (e < e1) {
            const long long n = e / V, v = e - n * V;
            a[u].load(x + e * ldx + cg * 8);
#pragma unroll
            for (int k = 0; k < 8; ++k) dd[u][k] = c0 + k < C ? dlog[(n * C + c0 + k) * V + v] : 0.f;
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const long long e = eb + u * lanes_v;
          if (e >= e1) break;
          const long long n = e / V;
          float xv[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) xv[j] = dscale ? a[u].get(j) * dscale[n * Cin + cg * 8 + j] : a[u].get(j);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float d = dd[u][k];
            bacc[k] += d;
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[k][j] = fmaf(d, xv[j], acc[k][j]);
          }
        }
      }
    }
    if (C8p <= 32) {
      // power-of-two channel groups: shuffle tree over the voxel lanes of each wave (fixed order), then
      // the 4 waves in order through LDS (the serial 64-lane LDS sweep per class cost ~2 us per block)
      for (int o = 32; o >= C8p; o >>= 1) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          bacc[k] += __shfl_down(bacc[k], o, 64);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[k][j] += __shfl_down(acc[k][j], o, 64);
        }
      }
      const int lane = tid & 63, wave = tid >> 6;
      for (int k = 0; k < 8 && c0 + k < C; ++k) {
        __syncthreads();
        if (lane < C8p) {
#pragma unroll
          for (int j = 0; j < 8; ++j) red[(wave * C8p + lane) * 8 + j] = acc[k][j];
          if (lane == 0) red[4 * 32 * 8 + wave] = bacc[k];
        }
        __syncthreads();
        for (int ci = tid; ci < Cin; ci += 256) {
          const int g = ci >> 3, j = ci & 7;
          float sacc = 0.f;
#pragma unroll
          for (int w = 0; w < 4; ++w) sacc += red[(w * C8p + g) * 8 + j];
          part[(long long)blockIdx.x * npairs + (c0 + k) * Cin + ci] = sacc;
        }
        if (tid == 0) {
          float sacc = 0.f;
#pragma unroll
          for (int w = 0; w < 4; ++w) sacc += red[4 * 32 * 8 + w];
          part[(long long)blockIdx.x * npairs + C * Cin + c0 + k] = sacc;
        }
      }
      continue;
    }
    for (int k = 0; k < 8 && c0 + k < C; ++k) {
      __syncthreads();
#pragma unroll
      for (int j = 0; j < 8; ++j) red[tid * 8 + j] = acc[k][j];
      __syncthreads();
      for (int ci = tid; ci < Cin; ci += 256) {
        const int g = ci >> 3, j = ci & 7;
        float sacc = 0.f;
        for (int l = 0; l < lanes_v; ++l) sacc += red[(l * C8 + g) * 8 + j];
        part[(long long)blockIdx.x * npairs + (c0 + k) * Cin + ci] = sacc;
      }
      __syncthreads();
      red[tid] = (cg == 0 && vl < lanes_v) ? bacc[k] : 0.f;
      __syncthreads();
      if (tid == 0) {
        float sacc = 0.f;
        for (int l = 0; l < lanes_v; ++l) sacc += red[l * C8];
        part[(long long)blockIdx.x * npairs + C * Cin + c0 + k] = sacc;
      }
    }
  }
}

// one wave per output (C*Cin weights + C biases): lanes stride over the block
// partials, fixed shuffle tree -> deterministic, 64 loads in flight per output
__global__ void head_wgrad_reduce(const float* __restrict__ part, int nblk, int C, int Cin, float* __restrict__ gW,
                                  float* __restrict__ gb, int accumulate) {
  const int npairs = C * Cin + C;
  const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (p >= npairs) return;
  float a = 0.f;
  for (int b = lane; b < nblk; b += 64) a += part[(long long)b * npairs + p];
  a = wave_sum(a);
  if (lane == 0) {
    float* dst = p < C * Cin ? gW + p : gb + (p - C * Cin);
    *dst = accumulate ? *dst + a : a;
  }
}

// ----------------------------------------------------------------- losses
struct LossCfg {
  int type;             // 0 = dice/ce family, 1 = tversky, 2 = focal (alpha = gamma; region weight 0)
  float dice_w, ce_w;   // weights of the region term and the CE term
  float smooth, alpha, beta;
  int include_bg;
  const float* cw;      // CE class weights [C] or null
};

// Label validity (the reference raises in F.one_hot / cross_entropy on a label outside [0, C)): such a
// voxel contributes nothing and is counted; the finalize pass then makes the loss NaN and publishes the
// count at coef[2NC+1] for the host to raise on.  Pure CE (region weight 0) skips torch's default
// ignore_index -100 without counting it, as nn.CrossEntropyLoss does.  Focal (type 2) skips it too: the
// reference's F.cross_entropy(reduction='none') gives 0 there (losses.py:116), and its .mean() still counts
// the voxel, so an ignored focal voxel adds 1 to the CE denominator and nothing else.
__device__ __forceinline__ int label_state(int y, int C, const LossCfg& cfg) {
  if ((unsigned)y < (unsigned)C) return 0;                 // valid
  return (y == -100 && ((cfg.type == 0 && cfg.dice_w == 0.f) || cfg.type == 2)) ? 1 : 2;   // 1 ignored, 2 invalid
}

// One voxel's contribution to the loss statistics: softmax p over its C logits z, Sum p / Sum p*t / Sum t per
// class and the (class-weighted / focal) CE term.  Shared by loss_stats_kernel and the fused head + loss
// forward so both give the same bits.  y must be a valid label.
template <int NC>
__device__ __forceinline__ void loss_voxel_stats(const float* z, int C, int y, const LossCfg& cfg, float* P, float* I,
                                                 float* Tc, float& ce, float& cden) {
  float mx = -INFINITY;
#pragma unroll
  for (int c = 0; c < NC; ++c)
    if (c < C) mx = fmaxf(mx, z[c]);
  float se = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c)
    if (c < C) se += expf(z[c] - mx);
  const float lse = mx + logf(se);
  const float inv = 1.f / se;
  float zy = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c)
    if (c < C) {
      const float p = expf(z[c] - mx) * inv;
      P[c] += p;
      if (c == y) {
        I[c] += p;
        Tc[c] += 1.f;
        zy = z[c];
      }
    }
  const float wy = cfg.cw ? cfg.cw[y] : 1.f;
  if (cfg.type == 2) {   // focal (losses.py:116-121): (1 - exp(-ce_i))^gamma * ce_i, plain mean over voxels
    const float cei = wy * (lse - zy);
    const float pt = expf(-cei);
    ce += powf(1.f - pt, cfg.alpha) * cei;
    cden += 1.f;
  } else {
    ce = fmaf(wy, lse - zy, ce);
    cden += wy;
  }
}

// One voxel's dloss/dlogits (before the output-gradient scale): d = p (dp - Sum p dp) + ce_scale w_y (p - t),
// dp = a t + b from the finalize pass's per-(n,c) coefficients cf = coef + 2 n C.  y must be valid.
template <int NC>
__device__ __forceinline__ void loss_voxel_grad(const float* z, int C, int y, const LossCfg& cfg,
                                                const float* __restrict__ cf, float ces, float* d) {
  float p[NC];
  float mx = -INFINITY;
#pragma unroll
  for (int c = 0; c < NC; ++c)
    if (c < C) mx = fmaxf(mx, z[c]);
  float se = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c)
    if (c < C) {
      p[c] = expf(z[c] - mx);
      se += p[c];
    }
  const float inv = 1.f / se;
  float wy = cfg.cw ? cfg.cw[y] : 1.f;
  if (cfg.type == 2) {   // focal: d f_i / d ce_i = gamma (1-pt)^(gamma-1) pt ce_i + (1-pt)^gamma, ce_i = w_y (lse - z_y)
    float zy = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (c < C && c == y) zy = z[c];
    const float cei = wy * (mx + logf(se) - zy);
    const float pt = expf(-cei), q = 1.f - pt, gm = cfg.alpha;
    const float dfd = (q > 0.f ? gm * powf(q, gm - 1.f) * pt * cei : 0.f) + powf(q, gm);
    wy *= dfd;
  }
  float dp[NC];
  float sacc = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c)
    if (c < C) {
      p[c] *= inv;
      const float t = c == y ? 1.f : 0.f;
      dp[c] = cf[2 * c] * t + cf[2 * c + 1];
      sacc = fmaf(p[c], dp[c], sacc);
    }
#pragma unroll
  for (int c = 0; c < NC; ++c)
    if (c < C) {
      const float t = c == y ? 1.f : 0.f;
      d[c] = p[c] * (dp[c] - sacc) + ces * wy * (p[c] - t);
    }
}

// per (n, chunk): [P_c][I_c][T_c] (3C) + ce_num + ce_den + invalid-label count
template <typename LT, int CC>
__global__ __launch_bounds__(256) void loss_stats_kernel(const float* __restrict__ logits, const LT* __restrict__ labels, int Crt,
                                  long long V, long long vpc, LossCfg cfg, float* __restrict__ part) {
  // CC > 0: class count known at compile time (U voxels in flight); CC = 0: runtime C, one voxel at a time
  const int C = CC > 0 ? CC : Crt;
  constexpr int NC = CC > 0 ? CC : CMAX;
  const int n = blockIdx.y, chunk = blockIdx.x, nchunk = gridDim.x;
  float P[NC], I[NC], Tc[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) P[c] = I[c] = Tc[c] = 0.f;
  float ce = 0.f, cden = 0.f, bad = 0.f;
  const long long v0 = (long long)chunk * vpc;
  long long v1 = v0 + vpc;
  if (v1 > V) v1 = V;
  const float* L = logits + (long long)n * C * V;
  // U voxels per thread per step: their C logits and labels are loaded before any is consumed
  constexpr int U = CC > 0 ? 4 : 1;
  for (long long vb = v0 + threadIdx.x; vb < v1; vb += U * blockDim.x) {
  float zu[U][NC];
  int yu[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long v = vb + u * blockDim.x;
    if (v < v1) {
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (c < C) zu[u][c] = L[c * V + v];
      yu[u] = (int)labels[(long long)n * V + v];
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (vb + u * blockDim.x >= v1) break;
    const int y = yu[u];
    const int ls = label_state(y, C, cfg);
    if (ls) {
      bad += ls == 2 ? 1.f : 0.f;
      if (ls == 1 && cfg.type == 2) cden += 1.f;   // focal: ignored voxel, counted by the mean
      continue;
    }
    loss_voxel_stats<NC>(zu[u], C, y, cfg, P, I, Tc, ce, cden);
  }
  }
  __shared__ float red[4][3 * CMAX + 3];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int c = 0; c < C; ++c) {
    float a = wave_sum(P[c]), b = wave_sum(I[c]), d = wave_sum(Tc[c]);
    if (lane == 0) {
      red[wave][c] = a;
      red[wave][C + c] = b;
      red[wave][2 * C + c] = d;
    }
  }
  {
    float a = wave_sum(ce), b = wave_sum(cden), d = wave_sum(bad);
    if (lane == 0) {
      red[wave][3 * C] = a;
      red[wave][3 * C + 1] = b;
      red[wave][3 * C + 2] = d;
    }
  }
  __syncthreads();
  const int nv = 3 * C + 3;
  for (int k = threadIdx.x; k < nv; k += blockDim.x)
    part[((long long)n * nchunk + chunk) * nv + k] = red[0][k] + red[1][k] + red[2][k] + red[3][k];
}

// one block: loss scalar + per-(n,c) dp coefficients (dp = a*t + b) + ce scale
// 1024 threads.  Phase 1: wave w sums quantity (n, q) over the chunks (lanes
// stride the chunks, fixed fp64 shuffle tree).  Phase 2: thread e = (n, c)
// forms the region term and its gradient coefficients.  Phase 3: thread 0
// adds the N*C region terms and the CE sums in index order.
__global__ void loss_finalize_kernel(const float* __restrict__ part, int N, int C, int nchunk, LossCfg cfg,
                                     float* __restrict__ loss_out, float* __restrict__ coef) {
  extern __shared__ double S[];           // [N*nv] sums, then [N*C] region terms
  const int nv = 3 * C + 3;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwave = blockDim.x >> 6;
  for (int pr = wave; pr < N * nv; pr += nwave) {
    const int n = pr / nv, q = pr - n * nv;
    double a = 0.0;
    for (int k = lane; k < nchunk; k += 64) a += part[((long long)n * nchunk + k) * nv + q];
    a = wave_sum_d(a);
    if (lane == 0) S[pr] = a;
  }
  __syncthreads();
  double* R = S + N * nv;
  const int c0 = (cfg.type == 0 && !cfg.include_bg) ? 1 : 0;
  const double nterms = (double)N * (C - c0);
  for (int e = threadIdx.x; e < N * C; e += blockDim.x) {
    const int n = e / C, c = e - n * C;
    const double P = S[n * nv + c], I = S[n * nv + C + c], T = S[n * nv + 2 * C + c];
    double a = 0.0, b = 0.0, region = 0.0;
    const double s = cfg.smooth;
    if (c >= c0) {
      if (cfg.type == 0) {
        const double U = P + T;
        const double dice = (2.0 * I + s) / (U + s);
        region = 1.0 - dice;
        a = -(2.0 / (U + s)) / nterms;
        b = ((2.0 * I + s) / ((U + s) * (U + s))) / nterms;
      } else {
        const double fp = P - I, fn = T - I;
        const double num = I + s;
        const double den = I + cfg.alpha * fp + cfg.beta * fn + s;
        region = 1.0 - num / den;
        a = -((den - num * (1.0 - cfg.alpha - cfg.beta)) / (den * den)) / nterms;
        b = (num * cfg.alpha / (den * den)) / nterms;
      }
    }
    R[e] = region;
    coef[e * 2 + 0] = (float)(a * cfg.dice_w);
    coef[e * 2 + 1] = (float)(b * cfg.dice_w);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double r = 0.0, ce = 0.0, den = 0.0, bad = 0.0;
    for (int e = 0; e < N * C; ++e) r += R[e];
    for (int n = 0; n < N; ++n) {
      ce += S[n * nv + 3 * C];
      den += S[n * nv + 3 * C + 1];
      bad += S[n * nv + 3 * C + 2];
    }
    const double lv = cfg.dice_w * (r / nterms) + cfg.ce_w * (ce / den);
    loss_out[0] = bad > 0.0 ? __builtin_nanf("") : (float)lv;
    coef[2 * N * C] = (float)(cfg.ce_w / den);   // CE gradient scale
    coef[2 * N * C + 1] = (float)bad;            // labels outside [0, C): the host raises on a non-zero count
  }
}

// dlogits = gout * [ p*(dp - sum p dp) + ce_scale * w_y * (p - t) ]
template <typename LT, int CC>
__global__ __launch_bounds__(256) void loss_bwd_kernel(const float* __restrict__ logits, const LT* __restrict__ labels, int Crt, long long V,
                                int N, LossCfg cfg, const float* __restrict__ coef, const float* __restrict__ gout,
                                float gconst, float* __restrict__ dlogits) {
  // CC > 0: class count known at compile time (U voxels in flight); CC = 0: runtime C, one voxel at a time
  const int C = CC > 0 ? CC : Crt;
  constexpr int NC = CC > 0 ? CC : CMAX;
  const long long total = (long long)N * V;
  const float g = gout ? gout[0] * gconst : gconst;
  const float ces = coef[2 * N * C];
  // U voxels per thread (i, i + S, ...): logits and labels of all U loaded before any is consumed
  constexpr int U = CC > 0 ? 4 : 1;
  const long long S = (long long)gridDim.x * blockDim.x;
  for (long long ib = (long long)blockIdx.x * blockDim.x + threadIdx.x; ib < total; ib += U * S) {
  float zu[U][NC];
  int yu[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long i = ib + u * S;
    if (i < total) {
      const long long n = i / V, v = i - n * V;
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (c < C) zu[u][c] = logits[(n * C + c) * V + v];
      yu[u] = (int)labels[i];
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long i = ib + u * S;
    if (i >= total) break;
    const long long n = i / V, v = i - n * V;
    const int y = yu[u];
    if (label_state(y, C, cfg)) {     // ignored / invalid label: no gradient through this voxel
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (c < C) dlogits[(n * C + c) * V + v] = 0.f;
      continue;
    }
    float d[NC];
    loss_voxel_grad<NC>(zu[u], C, y, cfg, coef + (long long)n * C * 2, ces, d);
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (c < C) dlogits[(n * C + c) * V + v] = g * d[c];
  }
  }
}

// ------------------------------------------------ fused head + loss (training)
// The Trainer's fast path (Trainer.train_step with an engine model and a HIP loss): the 1x1 head, the loss
// statistics and, in the backward, dlogits + the head's data and weight gradients, without materialising
// logits or dlogits.  Unfused, the same work is head_fwd (x -> 42 MB fp32 logits at 96^3 B=2), loss_stats
// (logits), loss_bwd (logits -> dlogits), head_dgrad (dlogits -> dx), head_wgrad_partial (x, dlogits): five
// passes at ~2.3 TB/s, 260 us.  Fused: the forward reads x + labels; the backward reads x + labels and
// writes dx, recomputing the logits.
//
// The head's two small GEMMs run on the matrix cores in exact fp32 (v_mfma_f32_16x16x4_f32, an fp32 fma
// chain): a wave takes 16 voxels per step; lane l holds channels 8g..8g+7 (g = l >> 4) of voxel l & 15 from
// one coalesced 16-B load (a wave's load = 16 voxels x 64 B, contiguous).
//   logits^T = W . x^T   (A = W, B = x^T; MFMA kb sums channels 8g + kb over the lane groups g)
//       -> lane l holds classes 4g..4g+3 of voxel l & 15: softmax = 4 registers + two cross-group shuffles;
//   dx^T = W^T . dlogits^T   (B = the lane's own dlogits registers: MFMA kb sums class 4g + kb)
//       -> lane l holds dx channels 16t + 4g .. +3 of voxel l & 15 (one 8-B store per 16-channel tile t);
//   dW += dlogits x (fp32 FMAs in the load layout, the voxel's dlogits gathered with 8 shuffles).
// Channel / class orders inside the sums differ from the unfused kernels', so values agree to fp32 rounding.
template <typename T, int G>
struct HeadLoad {   // the lane's 8 channels 8g..8g+7 of one voxel (zero for groups g >= G or invalid voxels)
  V8<T> a;
  bool in;
  __device__ __forceinline__ void load(const T* __restrict__ x, int ldx, long long row, bool ok, int g) {
    in = ok && g < G;
    if (in) a.load(x + row * ldx + 8 * g);
    else a.zero();
  }
  // the deferred InstanceNorm + ReLU of the last decoder block: relu((x - mean) * rstd) rounded to T, the
  // same operations as in_relu_apply, so the values equal the materialised output bit for bit
  __device__ __forceinline__ void norm(const float* mu, const float* rs) {
    if (!in) return;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float h = (a.get(j) - mu[j]) * rs[j];
      a.set(j, h > 0.f ? h : 0.f);
    }
  }
};

// the lane's 8 channels' InstanceNorm statistics (sample n), or none
template <int G>
__device__ __forceinline__ bool head_norm_stats(const float* nmean, const float* nrstd, int n, int g, float* mu,
                                                float* rs) {
  constexpr int Cin = 8 * G;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mu[j] = (nmean && g < G) ? nmean[n * Cin + 8 * g + j] : 0.f;
    rs[j] = (nmean && g < G) ? nrstd[n * Cin + 8 * g + j] : 1.f;
  }
  return nmean != nullptr;
}

constexpr int HU = 4;   // 16-voxel tiles per wave step in the fused head + loss kernels

// The wave's step loop over [vb, v1) in strides of `step`: fetch(regs, labels, vb) issues one step's loads,
// body(regs, labels, vb) consumes them.  (Issuing step k + 1's loads before step k's body, two register sets,
// measured slower: statistics pass 83 -> 94 us at 96^3 B=2, the backward spilled.)
template <typename T, int G, typename F, typename B>
__device__ __forceinline__ void head_steps(F& fetch, B& body, long long vb, long long v1, long long step) {
  for (; vb < v1; vb += step) {
    HeadLoad<T, G> l[HU];
    int y[HU];
    fetch(l, y, vb);
    body(l, y, vb);
  }
}

template <int G>
__device__ __forceinline__ f32x4 head_logits_t(const float* wA, const float* xs, const float* bz) {
  f32x4 acc = {bz[0], bz[1], bz[2], bz[3]};
#pragma unroll
  for (int kb = 0; kb < 8; ++kb) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wA[kb], xs[kb], acc, 0, 0, 0);
  return acc;
}

// BFL (bf16 storage, no Dropout3d scale): the same logits from two bf16 MFMAs (K = 32 = the lane's 8 channels x
// 4 lane groups, the load layout as is), W split into bf16 hi + lo parts: x is exact in bf16 and the products
// are exact, so the logits keep ~2^-17 of W (fp32 accumulation in another order) -- 32 MFMA cycles per 16
// voxels instead of 256 for the eight fp32 16x16x4 steps.
__device__ __forceinline__ void head_w_split(const float* wA, bf16x8& wh, bf16x8& wl) {
#pragma unroll
  for (int kb = 0; kb < 8; ++kb) {
    const bf16_t h = (bf16_t)wA[kb];
    wh[kb] = h;
    wl[kb] = (bf16_t)(wA[kb] - (float)h);
  }
}
__device__ __forceinline__ f32x4 head_logits_bf(const bf16x8& wh, const bf16x8& wl, const bf16x8& xa,
                                                const float* bz) {
  f32x4 acc = {bz[0], bz[1], bz[2], bz[3]};
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, xa, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl, xa, acc, 0, 0, 0);
}

template <typename T, int G, typename LT, bool BFL = false>
__global__ __launch_bounds__(256) void head_loss_stats_kernel(const T* __restrict__ x, int ldx,
                                                              const float* __restrict__ nmean,
                                                              const float* __restrict__ nrstd,
                                                              const float* __restrict__ Wt,
                                                              const float* __restrict__ bias,
                                                              const float* __restrict__ dscale, int C,
                                                              const LT* __restrict__ labels, long long V,
                                                              long long vpc, LossCfg cfg, float* __restrict__ part) {
  constexpr int Cin = 8 * G;
  __shared__ float red[4][52];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, v16 = lane & 15, g = lane >> 4;
  const int n = blockIdx.y, chunk = blockIdx.x, nchunk = gridDim.x;
  float nmu[8], nrs[8];
  const bool donorm = head_norm_stats<G>(nmean, nrstd, n, g, nmu, nrs);
  float wA[8], sc[8], bz[4];
#pragma unroll
  for (int kb = 0; kb < 8; ++kb) {
    wA[kb] = (v16 < C && g < G) ? Wt[v16 * Cin + 8 * g + kb] : 0.f;
    sc[kb] = (dscale && g < G) ? dscale[n * Cin + 8 * g + kb] : 1.f;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) bz[r] = 4 * g + r < C ? bias[4 * g + r] : 0.f;
  bf16x8 wAh, wAl;
  if constexpr (BFL) head_w_split(wA, wAh, wAl);
  float P[4], I[4], Tc[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) P[r] = I[r] = Tc[r] = 0.f;
  float ce = 0.f, cden = 0.f, bad = 0.f;
  const long long v0 = (long long)chunk * vpc;
  const long long v1 = v0 + vpc < V ? v0 + vpc : V;
  const long long base = (long long)n * V;
  // HU tiles of 16 voxels per wave step, all their loads in flight before the first is used (one 16-B load
  // per lane and tile is too little memory parallelism on its own)
  auto fetch = [&](HeadLoad<T, G>(&lds_)[HU], int(&ys_)[HU], long long vb) {
#pragma unroll
    for (int u = 0; u < HU; ++u) {
      const long long v = vb + 16 * u + v16;
      lds_[u].load(x, ldx, base + v, v < v1, g);
      ys_[u] = v < v1 ? (int)labels[base + v] : 0;
    }
  };
  auto body = [&](HeadLoad<T, G>(&lds_)[HU], const int(&ys_)[HU], long long vb) {
  if (donorm) {
#pragma unroll
    for (int u = 0; u < HU; ++u) lds_[u].norm(nmu, nrs);
  }
#pragma unroll
  for (int u = 0; u < HU; ++u) {
    const long long v = vb + 16 * u + v16;
    const bool ok = v < v1;
    const HeadLoad<T, G>& ld = lds_[u];
    const int y = ys_[u];
    f32x4 acc;
    if constexpr (BFL) {
      acc = head_logits_bf(wAh, wAl, ld.a.v, bz);
    } else {
      float xs[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) xs[j] = dscale ? ld.a.get(j) * sc[j] : ld.a.get(j);
      acc = head_logits_t<G>(wA, xs, bz);
    }
    float z[4], e[4];
    float mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      z[r] = 4 * g + r < C ? acc[r] : -INFINITY;
      mx = fmaxf(mx, z[r]);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float se = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      e[r] = 4 * g + r < C ? expf(z[r] - mx) : 0.f;
      se += e[r];
    }
    se += __shfl_xor(se, 16, 64);
    se += __shfl_xor(se, 32, 64);
    const float lse = mx + logf(se), inv = 1.f / se;
    const int ls = ok ? label_state(y, C, cfg) : 1;
    if (ls == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = 4 * g + r;
        if (c < C) {
          const float p = e[r] * inv;
          P[r] += p;
          if (c == y) {
            I[r] += p;
            Tc[r] += 1.f;
          }
        }
      }
      if ((y >> 2) == g) {   // the lane holding class y adds the voxel's CE term
        float zy = z[0];
#pragma unroll
        for (int r = 1; r < 4; ++r)
          if ((y & 3) == r) zy = z[r];
        const float wy = cfg.cw ? cfg.cw[y] : 1.f;
        if (cfg.type == 2) {
          const float cei = wy * (lse - zy);
          const float pt = expf(-cei);
          ce += powf(1.f - pt, cfg.alpha) * cei;
          cden += 1.f;
        } else {
          ce = fmaf(wy, lse - zy, ce);
          cden += wy;
        }
      }
    } else if (ls == 2 && g == 0) {
      bad += 1.f;
    } else if (ls == 1 && ok && cfg.type == 2 && g == 0) {
      cden += 1.f;   // focal: ignored (-100) voxel, counted by the mean
    }
  }
  };
  head_steps<T, G>(fetch, body, v0 + wave * 16 * HU, v1, 64 * HU);
  // sums over the 16 voxel lanes of each group (fixed tree); lane 16g then holds classes 4g..4g+3
#pragma unroll
  for (int o = 1; o < 16; o <<= 1)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      P[r] += __shfl_xor(P[r], o, 64);
      I[r] += __shfl_xor(I[r], o, 64);
      Tc[r] += __shfl_xor(Tc[r], o, 64);
    }
  ce = wave_sum(ce);
  cden = wave_sum(cden);
  bad = wave_sum(bad);
  if (v16 == 0)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      red[wave][4 * g + r] = P[r];
      red[wave][16 + 4 * g + r] = I[r];
      red[wave][32 + 4 * g + r] = Tc[r];
    }
  if (lane == 0) {
    red[wave][48] = ce;
    red[wave][49] = cden;
    red[wave][50] = bad;
  }
  __syncthreads();
  const int nv = 3 * C + 3;
  for (int k = threadIdx.x; k < nv; k += blockDim.x) {
    const int src = k < 3 * C ? (k / C) * 16 + k % C : 48 + (k - 3 * C);
    part[((long long)n * nchunk + chunk) * nv + k] = red[0][src] + red[1][src] + red[2][src] + red[3][src];
  }
}

// wpart: per block [C*Cin + C] weight / bias gradient partials (head_wgrad_reduce sums them over the blocks)
template <typename T, int G, int NC, typename LT, bool DS, bool BFL = false>
__global__ __launch_bounds__(256, (NC <= 6 && sizeof(T) == 2) ? 2 : 1) void head_loss_bwd_kernel(const T* __restrict__ x, int ldx,
                                                            const float* __restrict__ nmean,
                                                            const float* __restrict__ nrstd,
                                                            const float* __restrict__ Wt,
                                                            const float* __restrict__ bias,
                                                            const float* __restrict__ dscale, int C,
                                                            const LT* __restrict__ labels, long long V, long long vpc,
                                                            LossCfg cfg, const float* __restrict__ coef,
                                                            const float* __restrict__ gout, float gconst,
                                                            T* __restrict__ dx, int lddx, float* __restrict__ wpart,
                                                            float* __restrict__ inpart) {
  constexpr int Cin = 8 * G, TN = (Cin + 15) / 16;
  static_assert(NC <= 8, "dlogits gather covers 8 classes");
  // G == 4: MFMA row r of dx tile t is channel 8 (r >> 2) + 4 t + (r & 3), so lane group g ends up holding the
  // gradient of channels 8g..8g+7 of its voxel -- the channels of its own feature load: one 16-B store per voxel
  // (two 8-B stores otherwise), and the InstanceNorm-backward partial sums below need no lane exchange
  constexpr bool PERM = (G == 4);
  if constexpr (!DS) dscale = nullptr;   // no Dropout3d scale: the compiler drops the scale registers
  auto dx_chan = [](int t, int r) { return PERM ? 8 * (r >> 2) + 4 * t + (r & 3) : 16 * t + r; };
  __shared__ float red[4][NC * Cin + NC];
  __shared__ float ired[4][2][Cin];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, v16 = lane & 15, g = lane >> 4;
  const int n = blockIdx.y, chunk = blockIdx.x, nchunk = gridDim.x;
  float nmu[8], nrs[8];
  const bool donorm = head_norm_stats<G>(nmean, nrstd, n, g, nmu, nrs);
  float wA[8], sc[8], bz[4], ca[4], cb[4];
#pragma unroll
  for (int kb = 0; kb < 8; ++kb) {
    wA[kb] = (v16 < C && g < G) ? Wt[v16 * Cin + 8 * g + kb] : 0.f;
    sc[kb] = (dscale && g < G) ? dscale[n * Cin + 8 * g + kb] : 1.f;
  }
  bf16x8 wAh, wAl;
  if constexpr (BFL) head_w_split(wA, wAh, wAl);
  // BFL, PERM: dx^T from bf16 MFMAs too.  Lane group g's k-slots 0..3 carry classes 4g..4g+3 (hi parts of dlogits),
  // slots 4..7 the same classes' lo parts; A = (W hi, W hi) then (W lo, W lo): two 16x16x32 MFMAs per 16-channel
  // tile give (Whi + Wlo)(dhi + dlo) with exact products and fp32 sums -- instead of four fp32 16x16x4 steps
  bf16x8 wDh[TN], wDl[TN];
  if constexpr (BFL && PERM) {
#pragma unroll
    for (int t = 0; t < TN; ++t)
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const int ci = dx_chan(t, v16), c = 4 * g + kb;
        const float w = (ci < Cin && c < C) ? Wt[c * Cin + ci] : 0.f;
        const bf16_t h = (bf16_t)w, l = (bf16_t)(w - (float)h);
        wDh[t][kb] = h;
        wDh[t][kb + 4] = h;
        wDl[t][kb] = l;
        wDl[t][kb + 4] = l;
      }
  }
  const float* cf = coef + (long long)n * C * 2;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int c = 4 * g + r;
    bz[r] = c < C ? bias[c] : 0.f;
    ca[r] = c < C ? cf[2 * c] : 0.f;
    cb[r] = c < C ? cf[2 * c + 1] : 0.f;
  }
  // dx^T A operand: row ci = 16t + v16, k-slot g <-> class 4g + kb
  float wD[TN][4], sd[TN][4];
#pragma unroll
  for (int t = 0; t < TN; ++t)
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      const int ci = dx_chan(t, v16), c = 4 * g + kb;
      wD[t][kb] = (ci < Cin && c < C) ? Wt[c * Cin + ci] : 0.f;
      const int co = dx_chan(t, 4 * g + kb);   // the output channel of register kb
      sd[t][kb] = (dscale && co < Cin) ? dscale[n * Cin + co] : 1.f;
    }
  const float gsc = gout ? gout[0] * gconst : gconst;
  const float ces = coef[2 * gridDim.y * C];
  float acc[NC][8], bacc[4];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[c][j] = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) bacc[r] = 0.f;
  // InstanceNorm-backward partials of the block feeding the head (inpart, PERM only): sums of g and g * h over
  // the block's voxels, g = dx * [h > 0], h the head's input feature (relu of the normalised value)
  float sg[8], sgx[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) sg[j] = sgx[j] = 0.f;
  const bool do_in = PERM && !DS && inpart != nullptr;   // (with the Dropout3d scale the registers run out)
  const long long v0 = (long long)chunk * vpc;
  const long long v1 = v0 + vpc < V ? v0 + vpc : V;
  const long long base = (long long)n * V;
  auto fetch = [&](HeadLoad<T, G>(&lds_)[HU], int(&ys_)[HU], long long vb) {
#pragma unroll
    for (int u = 0; u < HU; ++u) {
      const long long v = vb + 16 * u + v16;
      lds_[u].load(x, ldx, base + v, v < v1, g);
      ys_[u] = v < v1 ? (int)labels[base + v] : 0;
    }
  };
  auto body = [&](HeadLoad<T, G>(&lds_)[HU], const int(&ys_)[HU], long long vb) {
  if (donorm) {
#pragma unroll
    for (int u = 0; u < HU; ++u) lds_[u].norm(nmu, nrs);
  }
#pragma unroll
  for (int u = 0; u < HU; ++u) {
    const long long v = vb + 16 * u + v16;
    const bool ok = v < v1;
    const HeadLoad<T, G>& ld = lds_[u];
    const int y = ys_[u];
    float xs[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) xs[j] = dscale ? ld.a.get(j) * sc[j] : ld.a.get(j);
    f32x4 acc_l;
    if constexpr (BFL) acc_l = head_logits_bf(wAh, wAl, ld.a.v, bz);
    else acc_l = head_logits_t<G>(wA, xs, bz);
    float z[4], p[4];
    float mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      z[r] = 4 * g + r < C ? acc_l[r] : -INFINITY;
      mx = fmaxf(mx, z[r]);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float se = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      p[r] = 4 * g + r < C ? expf(z[r] - mx) : 0.f;
      se += p[r];
    }
    se += __shfl_xor(se, 16, 64);
    se += __shfl_xor(se, 32, 64);
    const float inv = 1.f / se;
    const int ls = ok ? label_state(y, C, cfg) : 1;
    float wy = (ls == 0 && cfg.cw) ? cfg.cw[y] : 1.f;
    if (cfg.type == 2) {   // focal: the lane group holding class y has z_y; every lane needs it
      float zc = z[0];
#pragma unroll
      for (int r = 1; r < 4; ++r)
        if ((y & 3) == r) zc = z[r];
      const float zy = __shfl(zc, ((y >> 2) & 3) * 16 + v16, 64);
      const float cei = wy * (mx + logf(se) - zy);
      const float pt = expf(-cei), q = 1.f - pt, gm = cfg.alpha;
      const float dfd = (q > 0.f ? gm * powf(q, gm - 1.f) * pt * cei : 0.f) + powf(q, gm);
      wy *= dfd;
    }
    float dp[4], sp = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      p[r] *= inv;
      const float t = 4 * g + r == y ? 1.f : 0.f;
      dp[r] = ca[r] * t + cb[r];
      sp = fmaf(p[r], dp[r], sp);
    }
    sp += __shfl_xor(sp, 16, 64);
    sp += __shfl_xor(sp, 32, 64);
    float d[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float t = 4 * g + r == y ? 1.f : 0.f;
      d[r] = (ls == 0 && 4 * g + r < C) ? gsc * (p[r] * (dp[r] - sp) + ces * wy * (p[r] - t)) : 0.f;
      bacc[r] += d[r];
    }
    // dx^T = W^T dlogits^T (exact fp32 MFMA), 4 channels of voxel v per lane and 16-channel tile
    if constexpr (PERM) {
      V8<T> dv;
      bf16x8 db;
      if constexpr (BFL) {
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) {
          const bf16_t h = (bf16_t)d[kb];
          db[kb] = h;
          db[kb + 4] = (bf16_t)(d[kb] - (float)h);
        }
      }
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        f32x4 o = {0.f, 0.f, 0.f, 0.f};
        if constexpr (BFL) {
          o = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wDh[t], db, o, 0, 0, 0);
          o = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wDl[t], db, o, 0, 0, 0);
        } else {
#pragma unroll
          for (int kb = 0; kb < 4; ++kb) o = __builtin_amdgcn_mfma_f32_16x16x4f32(wD[t][kb], d[kb], o, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) dv.set(4 * t + r, dscale ? o[r] * sd[t][r] : o[r]);
      }
      if (dx && ok) dv.store(dx + (base + v) * lddx + 8 * g);
      if (do_in && ok) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float h = ld.a.get(j);
          const float gg = h > 0.f ? dv.get(j) : 0.f;
          sg[j] += gg;
          sgx[j] = fmaf(gg, h, sgx[j]);
        }
      }
    } else
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) o = __builtin_amdgcn_mfma_f32_16x16x4f32(wD[t][kb], d[kb], o, 0, 0, 0);
      const int co = 16 * t + 4 * g;
      if (dx && ok && co < Cin) {
        T* dst = dx + (base + v) * lddx + co;
        if constexpr (sizeof(T) == 2) {
          typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
          bf16x4 w4;
#pragma unroll
          for (int r = 0; r < 4; ++r) w4[r] = (bf16_t)(dscale ? o[r] * sd[t][r] : o[r]);
          *reinterpret_cast<bf16x4*>(dst) = w4;
        } else {
          float4 w4;
          w4.x = dscale ? o[0] * sd[t][0] : o[0];
          w4.y = dscale ? o[1] * sd[t][1] : o[1];
          w4.z = dscale ? o[2] * sd[t][2] : o[2];
          w4.w = dscale ? o[3] * sd[t][3] : o[3];
          *reinterpret_cast<float4*>(dst) = w4;
        }
      }
    }
    // dW[c][8g + j] += d[v][c] x[v][8g + j]: the voxel's dlogits of classes 0..NC-1 from lanes (c >> 2, v16)
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const float dc = __shfl(d[c & 3], (c >> 2) * 16 + v16, 64);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[c][j] = fmaf(dc, xs[j], acc[c][j]);
    }
  }
  };
  head_steps<T, G>(fetch, body, v0 + wave * 16 * HU, v1, 64 * HU);
  // fixed-order sums over the 16 voxel lanes of each group, then the 4 waves in order
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) {
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[c][j] += __shfl_xor(acc[c][j], o, 64);
#pragma unroll
    for (int r = 0; r < 4; ++r) bacc[r] += __shfl_xor(bacc[r], o, 64);
  }
  if (v16 == 0 && g < G)
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int j = 0; j < 8; ++j) red[wave][c * Cin + 8 * g + j] = acc[c][j];
  if (v16 == 0)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (4 * g + r < NC) red[wave][NC * Cin + 4 * g + r] = bacc[r];
  if (do_in) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sg[j] += __shfl_xor(sg[j], o, 64);
        sgx[j] += __shfl_xor(sgx[j], o, 64);
      }
    if (v16 == 0)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        ired[wave][0][8 * g + j] = sg[j];
        ired[wave][1][8 * g + j] = sgx[j];
      }
  }
  __syncthreads();
  const long long blk = (long long)n * nchunk + chunk;
  if (do_in && threadIdx.x < Cin) {   // in the layout of norm_pool.hip in_bwd_partial: [n][chunk][c][2]
    const int c = threadIdx.x;
    float* ip = inpart + (blk * Cin + c) * 2;
    ip[0] = ired[0][0][c] + ired[1][0][c] + ired[2][0][c] + ired[3][0][c];
    ip[1] = ired[0][1][c] + ired[1][1][c] + ired[2][1][c] + ired[3][1][c];
  }
  const int npairs = C * Cin + C;
  for (int k = threadIdx.x; k < npairs; k += blockDim.x) {
    const int src = k < C * Cin ? k : NC * Cin + (k - C * Cin);
    wpart[blk * npairs + k] = red[0][src] + red[1][src] + red[2][src] + red[3][src];
  }
}

// -------------------------------------------------------------- metric
// counts[0..C) intersection, [C..2C) pred count, [2C..3C) target count
template <typename LT>
__global__ void dice_counts_kernel(const float* __restrict__ logits, const LT* __restrict__ labels, int C, long long V,
                                   int N, unsigned long long* __restrict__ counts, LT* __restrict__ pred_out) {
  __shared__ unsigned int sc[3 * CMAX];
  for (int k = threadIdx.x; k < 3 * C; k += blockDim.x) sc[k] = 0;
  __syncthreads();
  const long long total = (long long)N * V;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long n = i / V, v = i - n * V;
    const float* L = logits + n * C * V;
    int best = 0;
    float bv = L[v];
    for (int c = 1; c < C; ++c) {
      const float z = L[c * V + v];
      if (z > bv || (z != z && bv == bv)) {  // first maximum; NaN counts as maximal (torch.argmax)
        bv = z;
        best = c;
      }
    }
    const int y = (int)labels[i];
    if (pred_out) pred_out[i] = (LT)best;
    atomicAdd(&sc[C + best], 1u);
    if (y >= 0 && y < C) {
      atomicAdd(&sc[2 * C + y], 1u);
      if (y == best) atomicAdd(&sc[y], 1u);
    }
  }
  __syncthreads();
  for (int k = threadIdx.x; k < 3 * C; k += blockDim.x)
    if (sc[k]) atomicAdd(&counts[k], (unsigned long long)sc[k]);
}

template <typename PT, typename LT>
__global__ void dice_counts_idx_kernel(const PT* __restrict__ pred, const LT* __restrict__ labels, int C,
                                       long long total, unsigned long long* __restrict__ counts) {
  __shared__ unsigned int sc[3 * CMAX];
  for (int k = threadIdx.x; k < 3 * C; k += blockDim.x) sc[k] = 0;
  __syncthreads();
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int p = (int)pred[i], y = (int)labels[i];
    if (p >= 0 && p < C) atomicAdd(&sc[C + p], 1u);
    if (y >= 0 && y < C) {
      atomicAdd(&sc[2 * C + y], 1u);
      if (y == p) atomicAdd(&sc[y], 1u);
    }
  }
  __syncthreads();
  for (int k = threadIdx.x; k < 3 * C; k += blockDim.x)
    if (sc[k]) atomicAdd(&counts[k], (unsigned long long)sc[k]);
}

// ------------------------------------------------------------------ AdamW (AdamHyper, adamw_load, adamw_one:
// mmseg_common.h)
__global__ void adamw_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                             float* __restrict__ v, long long n, AdamHyper hv, const AdamHyper* __restrict__ hp,
                             const float* __restrict__ skip) {
#pragma clang fp contract(off)
  AdamHyper h;
  if (!adamw_load(hv, hp, skip, h)) return;
  const float decay = h.decay, omb1 = h.omb1, beta2 = h.beta2, omb2 = h.omb2, eps = h.eps, step_size = h.step_size,
              bc2_sqrt = h.bc2_sqrt;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float pv = p[i];
    const float gv = g[i];
    pv = pv * decay;                          // param.mul_(1 - lr * wd)
    float mv = m[i];
    mv = omb1 < 0.5f ? mv + omb1 * (gv - mv)  // exp_avg.lerp_(grad, 1 - beta1)
                     : gv - (gv - mv) * (1.f - omb1);
    float vv = v[i];
    vv = vv * beta2 + (omb2 * gv) * gv;       // exp_avg_sq.mul_(b2).addcmul_(g, g, 1 - b2)
    const float denom = sqrtf(vv) / bc2_sqrt + eps;
    pv = pv + (-step_size) * (mv / denom);
    p[i] = pv;
    m[i] = mv;
    v[i] = vv;
  }
}

// float4 lanes, two vectors in flight per thread (the scalar kernel above kept one 4-B load of each stream in
// flight per thread: 177 us for the DualEncoder's 20 M parameters).  Same per-element arithmetic (bitwise equal).
// ntail (< 4): the scalar elements after the last float4, done by block 0's first threads (the same
// per-element operations as adamw_kernel, so bitwise its results) -- no second launch per step for them.
__global__ __launch_bounds__(256) void adamw4_kernel(float4* __restrict__ p, const float4* __restrict__ g,
                                                     float4* __restrict__ m, float4* __restrict__ v, long long n4,
                                                     AdamHyper hv, const AdamHyper* __restrict__ hp,
                                                     const float* __restrict__ skip, int ntail) {
  AdamHyper h;
  if (!adamw_load(hv, hp, skip, h)) return;
  if (blockIdx.x == 0 && (int)threadIdx.x < ntail) {
    const long long k = 4 * n4 + threadIdx.x;
    float* ps = reinterpret_cast<float*>(p);
    float* ms = reinterpret_cast<float*>(m);
    float* vs = reinterpret_cast<float*>(v);
    float pv = ps[k], mv = ms[k], vv = vs[k];
    adamw_one(pv, reinterpret_cast<const float*>(g)[k], mv, vv, h);
    ps[k] = pv;
    ms[k] = mv;
    vs[k] = vv;
  }
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += 2 * stride) {
    const long long i2 = i + stride;
    const bool two = i2 < n4;
    float4 pv[2], gv[2], mv[2], vv[2];
    pv[0] = p[i];
    gv[0] = g[i];
    mv[0] = m[i];
    vv[0] = v[i];
    if (two) {
      pv[1] = p[i2];
      gv[1] = g[i2];
      mv[1] = m[i2];
      vv[1] = v[i2];
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (u == 1 && !two) break;
      adamw_one(pv[u].x, gv[u].x, mv[u].x, vv[u].x, h);
      adamw_one(pv[u].y, gv[u].y, mv[u].y, vv[u].y, h);
      adamw_one(pv[u].z, gv[u].z, mv[u].z, vv[u].z, h);
      adamw_one(pv[u].w, gv[u].w, mv[u].w, vv[u].w, h);
      const long long k = u == 0 ? i : i2;
      p[k] = pv[u];
      m[k] = mv[u];
      v[k] = vv[u];
    }
  }
}

int grid_for(long long total) {
  long long b = (total + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (int)b;
}

// MMSEG_HEAD_BF16 (default 1): the fused head + loss kernels' logits from bf16 hi + lo MFMAs (head_logits_bf);
// read per call, so A/B runs and tests can flip it in-process
bool head_bf16() {
  const char* e = getenv("MMSEG_HEAD_BF16");
  return e ? atoi(e) != 0 : true;
}

// 1,728 voxels: 1,024 blocks at 96^3 B=2, one full round of the fused statistics kernel (118 VGPRs: 4 blocks per
// CU); 2,048 left 864 blocks, 3-4 per CU (83 -> 75 us, tools/headbench.py)
int loss_vpc() { return 1728; }

int loss_chunks(long long V, long long* vpc) {
  const int want = loss_vpc();
  long long nch = (V + want - 1) / want;
  if (nch > 4096) nch = 4096;
  if (nch < 1) nch = 1;
  *vpc = (V + nch - 1) / nch;
  return (int)((V + *vpc - 1) / *vpc);
}

// Voxel chunks of the fused head + loss backward, its own grid: 249 VGPRs hold it at two waves per SIMD, so
// 3,456 voxels (512 blocks at 96^3 B=2) are one full round of 256 CUs x 2 blocks; the statistics pass's 1,024 /
// 864 blocks took two (114 / 129 -> 110 us, tools/headbench.py).
int head_bwd_chunks(long long V, long long* vpc) {
  const int want = 3456;
  long long nch = (V + want - 1) / want;
  if (nch > 4096) nch = 4096;
  if (nch < 1) nch = 1;
  *vpc = (V + nch - 1) / nch;
  return (int)((V + *vpc - 1) / *vpc);
}

// Dispatch over the compile-time variants: storage type, 8-channel groups G (Cin = 8 G: 8 for the tiny test
// networks, 16, 32 for the configs' heads), class slots NC >= C (<= 8), label type.
template <typename F>
bool head_loss_dispatch(int C, int Cin, int dtype, int label_bytes, F&& f) {
  auto with_lt = [&](auto tag, auto g_c, auto nc_c) {
    if (label_bytes == 8) f(tag, g_c, nc_c, int64_t{});
    else f(tag, g_c, nc_c, uint8_t{});
    return true;
  };
  auto with_nc = [&](auto tag, auto g_c) {
    if (C <= 3) return with_lt(tag, g_c, std::integral_constant<int, 3>{});
    if (C <= 6) return with_lt(tag, g_c, std::integral_constant<int, 6>{});
    if (C <= 8) return with_lt(tag, g_c, std::integral_constant<int, 8>{});
    return false;
  };
  auto with_g = [&](auto tag) {
    if (Cin == 8) return with_nc(tag, std::integral_constant<int, 1>{});
    if (Cin == 16) return with_nc(tag, std::integral_constant<int, 2>{});
    if (Cin == 32) return with_nc(tag, std::integral_constant<int, 4>{});
    return false;
  };
  return dtype == MMSEG_BF16 ? with_g(bf16_t{}) : with_g(float{});
}

}  // namespace

extern "C" {

int mmseg_pack_input(const float* x, int Ctot, int c0, int cnt, int N, long long V, void* out, int dtype,
                     void* stream) {
  MMSEG_REQUIRE(cnt >= 1 && cnt <= 8, "pack_input: 1..8 channels per pack (got %d)", cnt);
  hipStream_t s = (hipStream_t)stream;
  const int grid = grid_for((long long)N * V);
  if (dtype == MMSEG_BF16)
    MMSEG_LAUNCH(pack_input_kernel<bf16_t>, dim3(grid), dim3(256), 0, s, x, Ctot, c0, cnt, V, N, (bf16_t*)out);
  else
    MMSEG_LAUNCH(pack_input_kernel<float>, dim3(grid), dim3(256), 0, s, x, Ctot, c0, cnt, V, N, (float*)out);
  return mmseg::check_launch("pack_input");
}

int mmseg_pack_input_compact(const float* x, int Ctot, int c0, int cnt, int N, long long V, void* out, int dtype,
                             void* stream) {
  MMSEG_REQUIRE(cnt >= 1 && cnt <= 4, "pack_input_compact: 1..4 channels (got %d)", cnt);
  hipStream_t s = (hipStream_t)stream;
  const int grid = grid_for((long long)N * V);
  if (dtype == MMSEG_BF16)
    MMSEG_LAUNCH(pack_input_compact_kernel<bf16_t>, dim3(grid), dim3(256), 0, s, x, Ctot, c0, cnt, V, N,
                       (bf16_t*)out);
  else
    MMSEG_LAUNCH(pack_input_compact_kernel<float>, dim3(grid), dim3(256), 0, s, x, Ctot, c0, cnt, V, N,
                       (float*)out);
  return mmseg::check_launch("pack_input_compact");
}

int mmseg_head_fwd(const void* x, int ldx, int Cin, const float* W, const float* b, const float* dscale, int C, int N,
                   long long V, float* logits, int dtype, void* stream) {
  MMSEG_REQUIRE(C >= 1 && C <= CMAX && Cin % 8 == 0, "head: 1 <= C <= %d, Cin%%8 == 0", CMAX);
  hipStream_t s = (hipStream_t)stream;
  const int ugrid = (int)ceil_div((long long)N * V, 256LL * 4);
  auto run_u = [&](auto tag, auto cg_c, auto cc_c) -> bool {
    using T = decltype(tag);
    constexpr int CG = decltype(cg_c)::value, CC = decltype(cc_c)::value;
    if (Cin != CG * 8 || C != CC) return false;
    if (CG == 6 && !dscale) {   // padded 48-channel rows: the tile-staged form
      const int tgrid = (int)std::min<long long>(ceil_div((long long)N * V, (long long)HT_V), 4096LL);
      MMSEG_LAUNCH((head_fwd_t_kernel<T, CG, CC>), dim3(tgrid), dim3(256), 0, s, (const T*)x, ldx, W, b, V, N,
                   logits);
      return true;
    }
    MMSEG_LAUNCH((head_fwd_u_kernel<T, CG, CC>), dim3(ugrid), dim3(256), 0, s, (const T*)x, ldx, W, b, dscale,
                       V, N, logits);
    return true;
  };
  // the configs' heads: 32 (UNet / DualEncoder) or 48 (SwinUNETR fs=48) input channels, 3 / 6 / 7 classes
  auto try_cc = [&](auto tag, auto cg_c) {
    return run_u(tag, cg_c, std::integral_constant<int, 3>{}) || run_u(tag, cg_c, std::integral_constant<int, 6>{}) ||
           run_u(tag, cg_c, std::integral_constant<int, 7>{});
  };
  auto try_u = [&](auto tag) {
    return try_cc(tag, std::integral_constant<int, 4>{}) || try_cc(tag, std::integral_constant<int, 6>{});
  };
  if (ldx % 8 == 0 && (dtype == MMSEG_BF16 ? try_u(bf16_t{}) : try_u(float{})))
    return mmseg::check_launch("head_fwd");
  const int grid = grid_for((long long)N * V);
  const size_t shm = (size_t)C * Cin * sizeof(float);
  if (dtype == MMSEG_BF16)
    MMSEG_LAUNCH(head_fwd_kernel<bf16_t>, dim3(grid), dim3(256), shm, s, (const bf16_t*)x, ldx, Cin, W, b, dscale,
                       C, V, N, logits);
  else
    MMSEG_LAUNCH(head_fwd_kernel<float>, dim3(grid), dim3(256), shm, s, (const float*)x, ldx, Cin, W, b, dscale,
                       C, V, N, logits);
  return mmseg::check_launch("head_fwd");
}

long long mmseg_head_ws_floats(int C, int Cin, int N, long long V) {
  const long long nblk = 2048;
  return nblk * (C * Cin + C);
}

int mmseg_head_bwd(const void* x, int ldx, int Cin, const float* W, const float* dscale, int C, int N, long long V,
                   const float* dlogits, void* dx, int lddx, float* gW, float* gb, float* ws, int accumulate, int dtype,
                   void* stream) {
  return mmseg_head_bwd_zw(x, ldx, Cin, W, dscale, C, N, V, dlogits, dx, lddx, Cin, gW, gb, ws, accumulate, dtype,
                           stream);
}

int mmseg_head_bwd_zw(const void* x, int ldx, int Cin, const float* W, const float* dscale, int C, int N, long long V,
                      const float* dlogits, void* dx, int lddx, int zcols, float* gW, float* gb, float* ws,
                      int accumulate, int dtype, void* stream) {
  MMSEG_REQUIRE(C >= 1 && C <= CMAX && Cin % 8 == 0 && Cin <= 2048, "head_bwd: shape");
  MMSEG_REQUIRE(zcols >= Cin && zcols % 8 == 0 && (!dx || zcols <= lddx), "head_bwd: zcols %d (Cin %d, lddx %d)",
                zcols, Cin, lddx);
  hipStream_t s = (hipStream_t)stream;
  const long long total = (long long)N * V;
#ifndef HEAD_DGRAD_GRID_CAP
#define HEAD_DGRAD_GRID_CAP 2048
#endif
  const int qgrid = std::min(grid_for(total * (zcols / 8)), HEAD_DGRAD_GRID_CAP);
  long long nblk = 2048;
  long long vpc = ((total + nblk - 1) / nblk + 63) / 64 * 64;
  nblk = (total + vpc - 1) / vpc;
  const size_t shm2 = 0;
  // weight-gradient partials first: dx may alias x (the engine reuses the feature buffer)
  if (dtype == MMSEG_BF16) {
    MMSEG_LAUNCH(head_wgrad_partial<bf16_t>, dim3((int)nblk), dim3(256), shm2, s, (const bf16_t*)x, ldx, dlogits,
                       dscale, C, Cin, V, N, vpc, ws);
    if (dx && C <= 8)
      MMSEG_LAUNCH((head_dgrad_g_kernel<bf16_t, 8>), dim3(qgrid), dim3(256), 0, s, dlogits, W, dscale, C, Cin, V, N,
                   (bf16_t*)dx, lddx, zcols / 8);
    else if (dx)
      MMSEG_LAUNCH((head_dgrad_g_kernel<bf16_t, CMAX>), dim3(qgrid), dim3(256), 0, s, dlogits, W, dscale, C, Cin, V,
                   N, (bf16_t*)dx, lddx, zcols / 8);
  } else {
    MMSEG_LAUNCH(head_wgrad_partial<float>, dim3((int)nblk), dim3(256), shm2, s, (const float*)x, ldx, dlogits,
                       dscale, C, Cin, V, N, vpc, ws);
    if (dx && C <= 8)
      MMSEG_LAUNCH((head_dgrad_g_kernel<float, 8>), dim3(qgrid), dim3(256), 0, s, dlogits, W, dscale, C, Cin, V, N,
                   (float*)dx, lddx, zcols / 8);
    else if (dx)
      MMSEG_LAUNCH((head_dgrad_g_kernel<float, CMAX>), dim3(qgrid), dim3(256), 0, s, dlogits, W, dscale, C, Cin, V,
                   N, (float*)dx, lddx, zcols / 8);
  }
  if (mmseg::check_launch("head_bwd")) return 1;
  MMSEG_LAUNCH(head_wgrad_reduce, dim3(ceil_div(C * Cin + C, 4)), dim3(256), 0, s, ws, (int)nblk, C, Cin, gW,
                     gb, accumulate);
  return mmseg::check_launch("head_wgrad_reduce");
}

long long mmseg_loss_ws_floats(int N, int C, long long V) {
  long long vpc;
  int nch = loss_chunks(V, &vpc);
  return (long long)N * nch * (3 * C + 3) + 2LL * N * C + 2;
}

// label_bytes: 8 (int64, the reference's dtype) or 1 (uint8)
int mmseg_loss_fwd(const float* logits, const void* labels, int label_bytes, int N, int C, long long V, int type,
                   float dice_w, float ce_w, float smooth, float alpha, float beta, int include_bg,
                   const float* class_w, float* loss_out, float* ws, void* stream) {
  MMSEG_REQUIRE(C >= 2 && C <= CMAX, "loss: 2 <= C <= %d", CMAX);
  MMSEG_REQUIRE(label_bytes == 8 || label_bytes == 1, "loss: labels must be int64 or uint8");
  LossCfg cfg{type, dice_w, ce_w, smooth, alpha, beta, include_bg, class_w};
  long long vpc;
  const int nch = loss_chunks(V, &vpc);
  float* part = ws;
  float* coef = ws + (long long)N * nch * (3 * C + 3);
  hipStream_t s = (hipStream_t)stream;
  auto stats = [&](auto lt, auto cc) {
    using LT = decltype(lt);
    MMSEG_LAUNCH((loss_stats_kernel<LT, decltype(cc)::value>), dim3(nch, N), dim3(256), 0, s, logits,
                       (const LT*)labels, C, V, vpc, cfg, part);
  };
  auto stats_c = [&](auto lt) {
    if (C == 3) stats(lt, std::integral_constant<int, 3>{});
    else if (C == 6) stats(lt, std::integral_constant<int, 6>{});
    else if (C == 7) stats(lt, std::integral_constant<int, 7>{});
    else stats(lt, std::integral_constant<int, 0>{});
  };
  if (label_bytes == 8) stats_c(int64_t{});
  else stats_c(uint8_t{});
  if (mmseg::check_launch("loss_stats")) return 1;
  const size_t shm = sizeof(double) * ((size_t)N * (3 * C + 3) + (size_t)N * C);
  MMSEG_REQUIRE(shm <= 64 * 1024, "loss: batch too large for the finalize pass (N=%d, C=%d)", N, C);
  MMSEG_LAUNCH(loss_finalize_kernel, dim3(1), dim3(1024), shm, s, part, N, C, nch, cfg, loss_out, coef);
  return mmseg::check_launch("loss_finalize");
}

// ------------------------------------------------ fused head + loss entries
int mmseg_head_loss_ok(int C, int Cin, int ldx, int dtype) {
  if (C < 2 || C > 8 || ldx % 8 != 0 || !(Cin == 8 || Cin == 16 || Cin == 32)) return 0;
  return (dtype == MMSEG_BF16 || dtype == MMSEG_F32) ? 1 : 0;
}

long long mmseg_head_loss_wpart_floats(int C, int Cin, int N, long long V) {
  long long vpc;
  const int nch = head_bwd_chunks(V, &vpc);
  return (long long)N * nch * (C * Cin + C);
}

int mmseg_head_loss_fwd(const void* x, int ldx, int Cin, const float* nmean, const float* nrstd, const float* W,
                        const float* b, const float* dscale, int C,
                        int N, long long V, const void* labels, int label_bytes, int type, float dice_w, float ce_w,
                        float smooth, float alpha, float beta, int include_bg, const float* class_w, float* loss_out,
                        float* ws, int dtype, void* stream) {
  MMSEG_REQUIRE(mmseg_head_loss_ok(C, Cin, ldx, dtype), "head_loss: unsupported shape (C=%d, Cin=%d, ldx=%d)", C,
                Cin, ldx);
  MMSEG_REQUIRE(label_bytes == 8 || label_bytes == 1, "head_loss: labels must be int64 or uint8");
  LossCfg cfg{type, dice_w, ce_w, smooth, alpha, beta, include_bg, class_w};
  long long vpc;
  const int nch = loss_chunks(V, &vpc);
  float* part = ws;
  float* coef = ws + (long long)N * nch * (3 * C + 3);
  hipStream_t s = (hipStream_t)stream;
  head_loss_dispatch(C, Cin, dtype, label_bytes, [&](auto tag, auto g_c, auto nc_c, auto lt) {
    using T = decltype(tag);
    using LT = decltype(lt);
    constexpr int G = decltype(g_c)::value, NC = decltype(nc_c)::value;
    (void)NC;                 // the statistics kernel does not depend on NC: one instance per (T, G, LT)
    mmseg::note_kernel("head_loss_stats_kernel");
    if (sizeof(T) == 2 && !dscale && head_bf16())
      MMSEG_LAUNCH((head_loss_stats_kernel<T, G, LT, sizeof(T) == 2>), dim3(nch, N), dim3(256), 0, s, (const T*)x,
                   ldx, nmean, nrstd, W, b, dscale, C, (const LT*)labels, V, vpc, cfg, part);
    else
      MMSEG_LAUNCH((head_loss_stats_kernel<T, G, LT>), dim3(nch, N), dim3(256), 0, s, (const T*)x, ldx, nmean,
                   nrstd, W, b, dscale, C, (const LT*)labels, V, vpc, cfg, part);
  });
  if (mmseg::check_launch("head_loss_stats")) return 1;
  const size_t shm = sizeof(double) * ((size_t)N * (3 * C + 3) + (size_t)N * C);
  MMSEG_REQUIRE(shm <= 64 * 1024, "head_loss: batch too large for the finalize pass (N=%d, C=%d)", N, C);
  MMSEG_LAUNCH(loss_finalize_kernel, dim3(1), dim3(1024), shm, s, part, N, C, nch, cfg, loss_out, coef);
  return mmseg::check_launch("loss_finalize");
}

// After mmseg_head_loss_fwd with the same ws.  dx may alias x (each voxel's features are read before its
// gradient is written); dx null skips the data gradient.  gW [C][Cin] / gb [C] (=, or += with accumulate).
int mmseg_head_loss_bwd_in(const void* x, int ldx, int Cin, const float* nmean, const float* nrstd, const float* W,
                           const float* b, const float* dscale, int C,
                           int N, long long V, const void* labels, int label_bytes, int type, float dice_w, float ce_w,
                           float smooth, float alpha, float beta, int include_bg, const float* class_w,
                           const float* gout, float gconst, const float* ws, void* dx, int lddx, float* gW, float* gb,
                           float* wpart, float* inpart, int accumulate, int dtype, void* stream);

int mmseg_head_loss_bwd(const void* x, int ldx, int Cin, const float* nmean, const float* nrstd, const float* W,
                        const float* b, const float* dscale, int C,
                        int N, long long V, const void* labels, int label_bytes, int type, float dice_w, float ce_w,
                        float smooth, float alpha, float beta, int include_bg, const float* class_w, const float* gout,
                        float gconst, const float* ws, void* dx, int lddx, float* gW, float* gb, float* wpart,
                        int accumulate, int dtype, void* stream) {
  return mmseg_head_loss_bwd_in(x, ldx, Cin, nmean, nrstd, W, b, dscale, C, N, V, labels, label_bytes, type, dice_w,
                                ce_w, smooth, alpha, beta, include_bg, class_w, gout, gconst, ws, dx, lddx, gW, gb,
                                wpart, nullptr, accumulate, dtype, stream);
}

int mmseg_head_loss_in_chunks(int C, int Cin, long long V) {
  if (Cin != 32 || C < 2 || C > 8) return 0;
  long long vpc;
  return head_bwd_chunks(V, &vpc);
}

int mmseg_head_loss_bwd_in(const void* x, int ldx, int Cin, const float* nmean, const float* nrstd, const float* W,
                           const float* b, const float* dscale, int C,
                           int N, long long V, const void* labels, int label_bytes, int type, float dice_w, float ce_w,
                           float smooth, float alpha, float beta, int include_bg, const float* class_w,
                           const float* gout, float gconst, const float* ws, void* dx, int lddx, float* gW, float* gb,
                           float* wpart, float* inpart, int accumulate, int dtype, void* stream) {
  MMSEG_REQUIRE(mmseg_head_loss_ok(C, Cin, ldx, dtype) && (dx == nullptr || lddx % 8 == 0),
                "head_loss_bwd: unsupported shape (C=%d, Cin=%d, ldx=%d, lddx=%d)", C, Cin, ldx, lddx);
  MMSEG_REQUIRE(!inpart || (mmseg_head_loss_in_chunks(C, Cin, V) > 0 && dx != nullptr && !dscale),
                "head_loss_bwd: InstanceNorm partials need Cin == 32, dx and no Dropout3d scale (C=%d, Cin=%d)", C,
                Cin);
  MMSEG_REQUIRE(!nmean || dx != x, "head_loss_bwd: with the deferred norm x is the pre-norm input the "
                "InstanceNorm backward still reads; dx must not alias it");
  LossCfg cfg{type, dice_w, ce_w, smooth, alpha, beta, include_bg, class_w};
  long long svpc, vpc;
  const int snch = loss_chunks(V, &svpc);   // the statistics pass's layout of ws
  const int nch = head_bwd_chunks(V, &vpc);
  const float* coef = ws + (long long)N * snch * (3 * C + 3);
  hipStream_t s = (hipStream_t)stream;
  head_loss_dispatch(C, Cin, dtype, label_bytes, [&](auto tag, auto g_c, auto nc_c, auto lt) {
    using T = decltype(tag);
    using LT = decltype(lt);
    constexpr int G = decltype(g_c)::value, NC = decltype(nc_c)::value;
    mmseg::note_kernel("head_loss_bwd_kernel");
    if (dscale)
      MMSEG_LAUNCH((head_loss_bwd_kernel<T, G, NC, LT, true>), dim3(nch, N), dim3(256), 0, s, (const T*)x, ldx,
                         nmean, nrstd, W, b, dscale, C, (const LT*)labels, V, vpc, cfg, coef, gout, gconst, (T*)dx,
                         lddx, wpart, inpart);
    else if (sizeof(T) == 2 && head_bf16())   // the statistics pass's logits (same switch)
      MMSEG_LAUNCH((head_loss_bwd_kernel<T, G, NC, LT, false, sizeof(T) == 2>), dim3(nch, N), dim3(256), 0, s,
                   (const T*)x, ldx, nmean, nrstd, W, b, dscale, C, (const LT*)labels, V, vpc, cfg, coef, gout,
                   gconst, (T*)dx, lddx, wpart, inpart);
    else
      MMSEG_LAUNCH((head_loss_bwd_kernel<T, G, NC, LT, false>), dim3(nch, N), dim3(256), 0, s, (const T*)x,
                         ldx, nmean, nrstd, W, b, dscale, C, (const LT*)labels, V, vpc, cfg, coef, gout, gconst,
                         (T*)dx, lddx, wpart, inpart);
  });
  if (mmseg::check_launch("head_loss_bwd")) return 1;
  MMSEG_LAUNCH(head_wgrad_reduce, dim3(ceil_div(C * Cin + C, 4)), dim3(256), 0, s, wpart, N * nch, C, Cin, gW,
                     gb, accumulate);
  return mmseg::check_launch("head_wgrad_reduce");
}

// Must follow mmseg_loss_fwd with the same ws.  gout (device scalar) may be null.
int mmseg_loss_bwd(const float* logits, const void* labels, int label_bytes, int N, int C, long long V, int type,
                   float dice_w, float ce_w, float smooth, float alpha, float beta, int include_bg,
                   const float* class_w, const float* gout, float gconst, float* dlogits, const float* ws,
                   void* stream) {
  LossCfg cfg{type, dice_w, ce_w, smooth, alpha, beta, include_bg, class_w};
  long long vpc;
  const int nch = loss_chunks(V, &vpc);
  const float* coef = ws + (long long)N * nch * (3 * C + 3);
  hipStream_t s = (hipStream_t)stream;
  auto bwd = [&](auto lt, auto cc) {
    using LT = decltype(lt);
    constexpr int CC = decltype(cc)::value;
    const int grid = grid_for(CC > 0 ? ceil_div((long long)N * V, 4) : (long long)N * V);
    MMSEG_LAUNCH((loss_bwd_kernel<LT, CC>), dim3(grid), dim3(256), 0, s, logits, (const LT*)labels, C, V, N, cfg,
                       coef, gout, gconst, dlogits);
  };
  auto bwd_c = [&](auto lt) {
    if (C == 3) bwd(lt, std::integral_constant<int, 3>{});
    else if (C == 6) bwd(lt, std::integral_constant<int, 6>{});
    else if (C == 7) bwd(lt, std::integral_constant<int, 7>{});
    else bwd(lt, std::integral_constant<int, 0>{});
  };
  if (label_bytes == 8) bwd_c(int64_t{});
  else bwd_c(uint8_t{});
  return mmseg::check_launch("loss_bwd");
}

// counts: 3*C uint64 (must be zeroed by the caller, accumulates); pred_out optional (same dtype as labels)
int mmseg_dice_counts(const float* logits, const void* labels, int label_bytes, int N, int C, long long V,
                      unsigned long long* counts, void* pred_out, void* stream) {
  MMSEG_REQUIRE(C >= 1 && C <= CMAX, "dice_counts: C <= %d", CMAX);
  hipStream_t s = (hipStream_t)stream;
  const int grid = grid_for((long long)N * V) > 2048 ? 2048 : grid_for((long long)N * V);
  if (label_bytes == 8)
    MMSEG_LAUNCH(dice_counts_kernel<int64_t>, dim3(grid), dim3(256), 0, s, logits, (const int64_t*)labels, C, V,
                       N, counts, (int64_t*)pred_out);
  else
    MMSEG_LAUNCH(dice_counts_kernel<uint8_t>, dim3(grid), dim3(256), 0, s, logits, (const uint8_t*)labels, C, V,
                       N, counts, (uint8_t*)pred_out);
  return mmseg::check_launch("dice_counts");
}

// counts from class-index masks (DiceMetric.update(pred, target), metrics.py:42-67); int64 or uint8 masks
int mmseg_dice_counts_idx(const void* pred, int pred_bytes, const void* labels, int label_bytes, long long total, int C,
                          unsigned long long* counts, void* stream) {
  MMSEG_REQUIRE(C >= 1 && C <= CMAX && (pred_bytes == 8 || pred_bytes == 1) && (label_bytes == 8 || label_bytes == 1),
                "dice_counts_idx: bad args");
  hipStream_t s = (hipStream_t)stream;
  const int grid = grid_for(total) > 2048 ? 2048 : grid_for(total);
#define DCI(PT, LT) \
  MMSEG_LAUNCH((dice_counts_idx_kernel<PT, LT>), dim3(grid), dim3(256), 0, s, (const PT*)pred, (const LT*)labels, C, total, counts)
  if (pred_bytes == 8 && label_bytes == 8) DCI(int64_t, int64_t);
  else if (pred_bytes == 8) DCI(int64_t, uint8_t);
  else if (label_bytes == 8) DCI(uint8_t, int64_t);
  else DCI(uint8_t, uint8_t);
#undef DCI
  return mmseg::check_launch("dice_counts_idx");
}

static int adamw_launch(float* p, const float* g, float* m, float* v, long long n, const AdamHyper& hv,
                        const AdamHyper* hp, const float* skip, hipStream_t stream) {
  const bool vec = ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(m) |
                     reinterpret_cast<uintptr_t>(v)) & 15) == 0;
  if (vec && n >= 4) {
    const long long n4 = n / 4;
    long long b4 = (n4 + 511) / 512;   // 2 float4 per thread
    if (b4 > 8192) b4 = 8192;
    MMSEG_LAUNCH(adamw4_kernel, dim3((int)b4), dim3(256), 0, stream, reinterpret_cast<float4*>(p),
                       reinterpret_cast<const float4*>(g), reinterpret_cast<float4*>(m), reinterpret_cast<float4*>(v),
                       n4, hv, hp, skip, (int)(n % 4));
    return mmseg::check_launch("adamw");
  }
  const int grid = grid_for(n) > 4096 ? 4096 : grid_for(n);
  MMSEG_LAUNCH(adamw_kernel, dim3(grid), dim3(256), 0, stream, p, g, m, v, n, hv, hp, skip);
  return mmseg::check_launch("adamw");
}

int mmseg_adamw(float* p, const float* g, float* m, float* v, long long n, float lr, float beta1, float beta2,
                float eps, float wd, int step, const float* skip, void* stream) {
  MMSEG_REQUIRE(step >= 1, "adamw: step counts from 1");
  return adamw_launch(p, g, m, v, n, adamw_hyper(lr, beta1, beta2, eps, wd, step), nullptr, skip,
                      (hipStream_t)stream);
}

int mmseg_adamw_hyper(float lr, float beta1, float beta2, float eps, float wd, int step, float* hyper) {
  MMSEG_REQUIRE(step >= 1 && hyper != nullptr, "adamw_hyper: step >= 1 and a host buffer of 8 floats");
  const AdamHyper h = adamw_hyper(lr, beta1, beta2, eps, wd, step);
  memcpy(hyper, &h, sizeof(h));
  return 0;
}

int mmseg_adamw_dev(float* p, const float* g, float* m, float* v, long long n, const float* hyper, const float* skip,
                    void* stream) {
  MMSEG_REQUIRE(hyper != nullptr, "adamw_dev: hyper (8 device floats from mmseg_adamw_hyper) required");
  AdamHyper unused{};
  return adamw_launch(p, g, m, v, n, unused, reinterpret_cast<const AdamHyper*>(hyper), skip, (hipStream_t)stream);
}

}  // extern "C"
