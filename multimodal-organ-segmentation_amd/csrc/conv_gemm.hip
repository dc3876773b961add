// Implicit-GEMM convolution kernels on CDNA4 MFMA (gfx950).
//
// One kernel family covers every GEMM-shaped op of the UNet3D / DualEncoder
// training step (reference unet.py:26-27 Conv3d(3,pad 1), unet.py:95
// ConvTranspose3d(2,2), unet.py:163 / dual_encoder.py:75 1x1 Conv3d):
//
//   rows (M)  = voxels of a "row grid" (N x D x H x W, flattened)
//   cols (N)  = output channels (x 8 taps for the transposed conv)
//   K         = k-groups of 8 consecutive channels ("kgi"), each bound to a tap
//
// The A operand is gathered per lane straight from the NDHWC activation
// (8 contiguous channels = one 16 B bf16 / 32 B f32 load), with zero padding
// for out-of-volume taps.  The B operand is the weight tensor pre-packed as
// [KGp][Cpad][8] so that each lane's fragment is one contiguous vector.
//
// bf16: one v_mfma_f32_16x16x32_bf16 per k-step (lane l holds rows l&15,
//       k = 8*(l>>4)+j).
// f32 : eight v_mfma_f32_16x16x4f32 per k-step (exact fp32 FMA chain); lane
//       element j of k-group (l>>4) feeds MFMA j, so A and B agree on K order.
//
// wgrad (dW = sum over voxels) runs as a second kernel with K = voxels: both
// operands are staged through LDS transposed (channel-major) and reduced in a
// fixed-order split-K pass, so weight gradients are bitwise deterministic.
#include "mmseg_common.h"

#include <stdlib.h>

#include <algorithm>
#include <type_traits>
#include <cstdio>
#include <vector>

namespace {

// Tuning knobs for in-process A/B runs (tools/kbench.py); defaults are the shipped choice.
int knob(const char* name, int dflt) {
  const char* v = getenv(name);
  return v ? atoi(v) : dflt;
}

enum GatherMode { MODE_CONV3 = 0, MODE_POINT = 1, MODE_CONVT_FWD = 2, MODE_CONVT_DGRAD = 3 };

// Block timeline probe (diagnostics, built only with -DMMSEG_TIMING_PROBES; tools/convbench.py --probe).
// Per block b < PROBE_NB: [realtime start, realtime end, memtime start, memtime end, HW_ID, XCC_ID, -, -];
// then for blocks < 32, every wave's lane 0 records up to 64 memtime stamps (PROBE_T) at phase boundaries.
#ifdef MMSEG_TIMING_PROBES
constexpr int PROBE_NB = 16384;
__device__ long long* g_probe = nullptr;
__device__ __forceinline__ void probe_block(bool end) {
  long long* p = g_probe;
  if (p && threadIdx.x == 0 && blockIdx.x < PROBE_NB) {
    p += 8LL * blockIdx.x;
    p[end ? 1 : 0] = (long long)__builtin_amdgcn_s_memrealtime();
    p[end ? 3 : 2] = (long long)__builtin_amdgcn_s_memtime();
    if (!end) {
      p[4] = (long long)(unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
      p[5] = (long long)(unsigned)__builtin_amdgcn_s_getreg((15 << 11) | 20);   // HW_REG_XCC_ID
    }
  }
}
__device__ __forceinline__ void probe_stamp(int& k) {
  long long* p = g_probe;
  if (p && (threadIdx.x & 63) == 0 && blockIdx.x < 32 && k < 64)
    p[8LL * PROBE_NB + ((blockIdx.x * 16 + (threadIdx.x >> 6)) * 64) + k] = (long long)__builtin_amdgcn_s_memtime();
  ++k;
}
#define PROBE_BLOCK(e) probe_block(e)
#define PROBE_T() probe_stamp(probe_k)
#define PROBE_DECL() int probe_k = 0
#else
#define PROBE_BLOCK(e)
#define PROBE_T()
#define PROBE_DECL()
#endif

struct GemmArgs {
  const void* a;  int lda;   // A source (NDHWC)
  const void* b;             // packed weights [KGp][Cpad][8]
  const float* bias;         // per output channel, or null
  void* out;      int ldo;   // output (NDHWC) for ksplit == 1
  float* part;               // [ksplit][M][Ncols] fp32 partials for ksplit > 1
  int M, Ncols, Cpad, KG, cpg_shift;
  int D, H, W;               // row grid
  int ksplit, kg_per_split;  // k-groups per split (multiple of 4)
  int swz;                   // XCD-aware block remap
  float* stats;              // brick kernels, ksplit == 1: per-brick InstanceNorm partials (mean, M2), or null
  int kchunks;               // CONV3 brick kernels: 32-channel input chunks holding real channels (0 = all);
                             // the packed weights of the rest are zero (channel-padded K side), so they are skipped
  // deferred InstanceNorm + ReLU of the A source (brick5 only, mmseg_conv3_fwd_norm): A holds the PRE-norm
  // activation, the kernel stages relu((a - nmean[n][c]) * nrstd[n][c]) rounded to T (in_relu_apply's values)
  const float* nmean;
  const float* nrstd;
  // split output (mmseg_conv_gemm_split): columns >= split go to out2 (column - split, row pitch ldo2).  The
  // decoder's first-conv data gradient writes d(upsampled) and d(skip) as two dense tensors instead of one
  // [voxel][2F] tensor whose halves every later reader fetched at half a cache line per voxel.
  void* out2;
  int ldo2, split;
  // InstanceNorm-backward partials of the output (brick5 data gradient only, mmseg_conv3_dgrad_in): the output is
  // the gradient dy of an InstanceNorm + ReLU whose PRE-norm input is inx (pitch ldinx, statistics inmean /
  // inrstd [N][Ncols]); the kernel also writes inpart[n][block][col][2] = (sum g, sum g xhat), g = dy [xhat > 0]
  const void* inx;
  int ldinx;
  const float* inmean;
  const float* inrstd;
  float* inpart;
  int prio;   // (unused: the s_setprio experiments of round 3 measured +-2 % and were removed)
  // fp8 forward (brick6 F8, mmseg_conv3_fwd_fp8): b holds e4m3 weights w * s[co] (s = 448 / max |w[co]|), wdq[co] =
  // 1 / s[co] restores the scale in the epilogue; the staged activations are e4m3 at unit scale
  const float* wdq;
  // grouped launch (mmseg_conv_gemm_group, runtime-brick kernel only): the samples are grp_n-sample groups with
  // their own weights / bias -- group gi reads b + gi * w_gstride (elements) and bias + gi * b_gstride; the M
  // modality encoders' small levels run as ONE launch over M x N samples
  int grp_n;
  long long w_gstride;
  int b_gstride;
  // residual epilogue (MODE_POINT, ksplit 1, vector stores; mmseg_conv_gemm_res): out = round(round(acc + bias) +
  // res), the values of the GEMM followed by mmseg_add(res, out) -- a residual sum without its own pass (res may
  // alias out)
  const void* res;
  int ldres;
  // whole-row output hint (brick2 kernels; others ignore it): the last column tile also writes zeros into columns
  // [Ncols, zcols) (<= Ncols + BN) of the output rows -- SwinUNETR's 48 / 96-column outputs at pitch 64 / 128 are
  // then written in whole 128-B lines (partial-line writes ran at ~60 % of the whole-row rate, r05k)
  int zcols;
  // token-GEMM epilogue (MODE_POINT, ksplit 1, vector stores; mmseg_conv_gemm_gelu): epi 1 = GELU forward, out = h
  // (the pre-activation the backward reads) and aux_out = gelu(h); epi 2 = GELU backward, out = round(round(acc) *
  // gelu'(aux)) with aux = h -- the values of the GEMM followed by mmseg_gelu_fwd / mmseg_gelu_bwd (pitch ldo)
  int epi;
  const void* aux;
  void* aux_out;
};

// Output element (row voxel, column) of a GEMM (split-aware; split is a multiple of 8).
template <typename T>
__device__ __forceinline__ T* out_at(const GemmArgs& g, long long vox, int col) {
  if (g.out2 && col >= g.split) return reinterpret_cast<T*>(g.out2) + vox * g.ldo2 + (col - g.split);
  return reinterpret_cast<T*>(g.out) + vox * g.ldo + col;
}

// The deferred norm of 8 staged channels: relu((v - mu) * rs) rounded to T, in_relu_apply's operations.
template <typename T>
__device__ __forceinline__ void norm_relu8(V8<T>& v, const float* mu, const float* rs) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float h = (v.get(j) - mu[j]) * rs[j];
    v.set(j, h > 0.f ? h : 0.f);
  }
}

// 32-channel K chunks a CONV3 brick kernel iterates: all of the (power-of-two) A source's, or only the
// leading ones that hold real channels.
__host__ __device__ __forceinline__ int gemm_nchunk(const GemmArgs& g) {
  const int n = (8 << g.cpg_shift) / 32;
  return (g.kchunks > 0 && g.kchunks < n) ? g.kchunks : n;
}

// Per-brick InstanceNorm statistics of a staged output tile (fused into the
// brick conv epilogue, so the IN stats pass never re-reads the conv output).
// El: [rows][EP] staged outputs (already rounded to the storage type, i.e. the
// exact values InstanceNorm will read); channel c = tid % BN, voxel slices
// tid / BN.  Two passes over LDS (mean, then sum of squared deviations), fixed
// order -> deterministic.  out[(brick * C + col) * 2 + {0, 1}] = (mean, M2).
template <typename T, int BN>
__device__ __forceinline__ void brick_in_stats(const T* El, int EP, int rows, float* red, float* out, long long brick,
                                               int n0, int C) {
  constexpr int S = 256 / BN;
  const int tid = threadIdx.x, c = tid % BN, sl = tid / BN;
  float a = 0.f;
  for (int v = sl; v < rows; v += S) a += (float)El[v * EP + c];
  red[tid] = a;
  __syncthreads();
  if (tid < BN) {
    float t = 0.f;
    for (int k = 0; k < S; ++k) t += red[k * BN + tid];
    red[256 + tid] = t / (float)rows;
  }
  __syncthreads();
  const float mu = red[256 + c];
  float q = 0.f;
  for (int v = sl; v < rows; v += S) {
    const float d = (float)El[v * EP + c] - mu;
    q = fmaf(d, d, q);
  }
  __syncthreads();
  red[tid] = q;
  __syncthreads();
  if (tid < BN && n0 + tid < C) {
    float t = 0.f;
    for (int k = 0; k < S; ++k) t += red[k * BN + tid];
    float* o = out + (brick * C + n0 + tid) * 2;
    o[0] = red[256 + tid];
    o[1] = t;
  }
}

template <typename T>
__device__ __forceinline__ void mfma_step(f32x4& acc, const V8<T>& a, const V8<T>& b);

template <>
__device__ __forceinline__ void mfma_step<bf16_t>(f32x4& acc, const V8<bf16_t>& a, const V8<bf16_t>& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, b.v, acc, 0, 0, 0);
}
template <>
__device__ __forceinline__ void mfma_step<float>(f32x4& acc, const V8<float>& a, const V8<float>& b) {
#pragma unroll
  for (int j = 0; j < 8; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.v[j], b.v[j], acc, 0, 0, 0);
}

// Per-lane row descriptor.
struct RowInfo {
  long long m;        // row index (voxel in row grid); -1 if out of range
  long long base;     // CONV3/POINT: m ; CONVT: child base voxel in 2x grid
  uint32_t tmask;     // CONV3: valid taps
};

template <int MODE>
__device__ __forceinline__ RowInfo make_row(long long m, const GemmArgs& g) {
  RowInfo r;
  r.m = m < g.M ? m : -1;
  r.base = m;
  r.tmask = 0;
  if (r.m < 0) return r;
  // 32-bit index arithmetic: M < 2^31 (the host checks M * lda), and 64-bit divisions cost ~100 VALU each
  if (MODE == MODE_CONV3) {
    const unsigned mu = (unsigned)m;
    const unsigned t = mu / (unsigned)g.W, x = mu - t * (unsigned)g.W;
    const unsigned t2 = t / (unsigned)g.H, y = t - t2 * (unsigned)g.H;
    const unsigned z = t2 % (unsigned)g.D;
    r.tmask = tap_valid_mask((int)z, (int)y, (int)x, g.D, g.H, g.W);
  } else if (MODE == MODE_CONVT_DGRAD) {
    const unsigned mu = (unsigned)m;
    const unsigned t = mu / (unsigned)g.W, x = mu - t * (unsigned)g.W;
    const unsigned t2 = t / (unsigned)g.H, y = t - t2 * (unsigned)g.H;
    const unsigned n = t2 / (unsigned)g.D, z = t2 - n * (unsigned)g.D;
    const long long H2 = 2LL * g.H, W2 = 2LL * g.W, D2 = 2LL * g.D;
    r.base = (((long long)n * D2 + 2 * z) * H2 + 2 * y) * W2 + 2 * x;
  }
  return r;
}

// Voxel offset of tap t relative to the row voxel (CONV3) or child (CONVT).
template <int MODE>
__device__ __forceinline__ long long tap_offset(int t, const GemmArgs& g) {
  if (MODE == MODE_CONV3) {
    int dz, dy, dx;
    tap_delta(t, dz, dy, dx);
    return ((long long)dz * g.H + dy) * g.W + dx;
  } else {   // 32-bit: the child grid's voxel count is < 2^31 (host: M * lda)
    const int a = t >> 2, b = (t >> 1) & 1, c = t & 1;
    return (long long)(a * (4 * g.H * g.W) + b * (2 * g.W) + c);
  }
}

template <typename T, int MODE>
__device__ __forceinline__ void load_a(V8<T>& v, const RowInfo& r, int kgi, const GemmArgs& g) {
  const T* A = reinterpret_cast<const T*>(g.a);
  bool ok = r.m >= 0 && kgi < g.KG;
  long long vox = 0;
  int c8 = kgi;
  if (MODE == MODE_CONV3) {
    int t = kgi >> g.cpg_shift;
    c8 = kgi & ((1 << g.cpg_shift) - 1);
    ok = ok && ((r.tmask >> t) & 1u);
    if (ok) vox = r.base + tap_offset<MODE_CONV3>(t, g);
  } else if (MODE == MODE_CONVT_DGRAD) {
    int t = kgi >> g.cpg_shift;
    c8 = kgi & ((1 << g.cpg_shift) - 1);
    vox = r.base + tap_offset<MODE_CONVT_DGRAD>(t, g);
  } else {
    vox = r.base;
  }
  if (ok) v.load(A + vox * g.lda + c8 * 8);
  else v.zero();
}

template <typename T>
__device__ __forceinline__ void load_b(V8<T>& v, int kgi, int col, const GemmArgs& g) {
  const T* B = reinterpret_cast<const T*>(g.b);
  v.load(B + ((long long)kgi * g.Cpad + col) * 8);
}

// Child voxel (2x grid) of input voxel `row` for transposed-conv tap t (32-bit divisions, see make_row).
__device__ __forceinline__ long long convt_child(long long row, int t, const GemmArgs& g) {
  const unsigned mu = (unsigned)row;
  const unsigned q = mu / (unsigned)g.W, x = mu - q * (unsigned)g.W;
  const unsigned q2 = q / (unsigned)g.H, y = q - q2 * (unsigned)g.H;
  const unsigned n = q2 / (unsigned)g.D, z = q2 - n * (unsigned)g.D;
  return (((long long)n * 2 * g.D + 2 * z + (t >> 2)) * 2LL * g.H + 2 * y + ((t >> 1) & 1)) * 2LL * g.W + 2 * x +
         (t & 1);
}

// Block = WM x WN waves; wave tile = (RM*16) x (RN*16).
template <typename T, int MODE, int WM, int WN, int RM, int RN>
__global__ __launch_bounds__(256) void conv_gemm_kernel(GemmArgs g) {
  constexpr int BM = WM * RM * 16;
  constexpr int BN = WN * RN * 16;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int mt_n = (g.M + BM - 1) / BM, nt_n = (g.Ncols + BN - 1) / BN;
  const int tile = g.swz ? xcd_swizzle(blockIdx.x, mt_n * nt_n * g.ksplit) : (int)blockIdx.x;
  const int mt = tile % mt_n, nt = (tile / mt_n) % nt_n, ks = tile / (mt_n * nt_n);
  const long long m0 = (long long)mt * BM + wm * RM * 16;
  const int n0 = nt * BN + wn * RN * 16;
  const int kg_begin = ks * g.kg_per_split;
  int kg_end = kg_begin + g.kg_per_split;
  const int KGp = (g.KG + 3) & ~3;
  if (kg_end > KGp) kg_end = KGp;

  RowInfo rows[RM];
#pragma unroll
  for (int i = 0; i < RM; ++i) rows[i] = make_row<MODE>(m0 + i * 16 + (lane & 15), g);

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int kq = lane >> 4;
  V8<T> ac[RM], bc[RN], an[RM], bn[RN];
  int kgi = kg_begin + kq;
  if (kg_begin < kg_end) {
#pragma unroll
    for (int i = 0; i < RM; ++i) load_a<T, MODE>(ac[i], rows[i], kgi, g);
#pragma unroll
    for (int j = 0; j < RN; ++j) load_b<T>(bc[j], kgi, n0 + j * 16 + (lane & 15), g);
  }
  for (int kb = kg_begin; kb < kg_end; kb += 4) {
    const int kn = kb + 4;
    if (kn < kg_end) {
      const int kgn = kn + kq;
#pragma unroll
      for (int i = 0; i < RM; ++i) load_a<T, MODE>(an[i], rows[i], kgn, g);
#pragma unroll
      for (int j = 0; j < RN; ++j) load_b<T>(bn[j], kgn, n0 + j * 16 + (lane & 15), g);
    }
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) mfma_step<T>(acc[i][j], ac[i], bc[j]);
    if (kn < kg_end) {
#pragma unroll
      for (int i = 0; i < RM; ++i) ac[i] = an[i];
#pragma unroll
      for (int j = 0; j < RN; ++j) bc[j] = bn[j];
    }
  }

  // epilogue: C/D layout col = lane&15, row = (lane>>4)*4 + r
  T* O = reinterpret_cast<T*>(g.out);
  const int Cout = (MODE == MODE_CONVT_FWD) ? (g.Ncols >> 3) : g.Ncols;
  if (g.ksplit > 1) {
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int col = n0 + j * 16 + (lane & 15);
        if (col >= g.Ncols) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const long long row = m0 + i * 16 + (lane >> 4) * 4 + r;
          if (row < g.M) g.part[((long long)ks * g.M + row) * g.Ncols + col] = acc[i][j][r];
        }
      }
    return;
  }
  // stage the (BM x BN) tile through LDS so every lane stores 8 channels (16 B bf16) at once;
  // for the transposed conv an 8-column group is 8 channels of ONE child voxel (Cout % 8 == 0)
  constexpr int EPT = BN + 8;
  __shared__ __attribute__((aligned(16))) T El[BM * EPT];
  const long long mt0 = (long long)mt * BM;
  const int nt0 = nt * BN;
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      const int lc = wn * RN * 16 + j * 16 + (lane & 15);
      const int col = nt0 + lc;
      float bv = 0.f;
      if (g.bias && col < g.Ncols) bv = g.bias[MODE == MODE_CONVT_FWD ? col % Cout : col];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int lr = wm * RM * 16 + i * 16 + (lane >> 4) * 4 + r;
        El[lr * EPT + lc] = from_f<T>(acc[i][j][r] + bv);
      }
    }
  __syncthreads();
  constexpr int CG = BN / 8;
  const bool vec = g.ldo % 8 == 0 && g.Ncols % 8 == 0 && (reinterpret_cast<uintptr_t>(g.out) & 15) == 0;
  if (!vec) {   // odd strides: element-wise stores from the staged tile
    for (int e = threadIdx.x; e < BM * BN; e += 256) {
      const int lr = e / BN, lc = e % BN;
      const long long row = mt0 + lr;
      const int col = nt0 + lc;
      if (row >= g.M || col >= g.Ncols) continue;
      if (MODE == MODE_CONVT_FWD) {
        const int t = col / Cout, co = col - t * Cout;
        O[convt_child(row, t, g) * g.ldo + co] = El[lr * EPT + lc];
      } else {
        *out_at<T>(g, row, col) = El[lr * EPT + lc];
      }
    }
    return;
  }
  if constexpr (MODE == MODE_CONVT_FWD) {
    // a thread's 8-column group (tap t, channels co..co+7) is the same in every pass (256 % CG == 0) and its rows
    // step by 256 / CG: the child voxel's coordinates are decomposed once and then stepped, instead of three
    // runtime divisions per store (the epilogue was ~28 VALU per MFMA, r04i PMC)
    static_assert(256 % CG == 0, "fixed column group per thread");
    constexpr int LSTEP = 256 / CG;
    const int cg = threadIdx.x % CG;
    const int col = nt0 + cg * 8;
    if (col >= g.Ncols) return;
    const int t = col / Cout, co = col - t * Cout;
    const int tz = t >> 2, ty = (t >> 1) & 1, tx = t & 1;
    int lr = threadIdx.x / CG;
    const unsigned mu = (unsigned)(mt0 + lr);
    const unsigned q = mu / (unsigned)g.W, q2 = q / (unsigned)g.H;
    int x = (int)(mu - q * (unsigned)g.W), y = (int)(q - q2 * (unsigned)g.H);
    int n = (int)(q2 / (unsigned)g.D), z = (int)(q2 - (unsigned)n * (unsigned)g.D);
    const long long W2 = 2LL * g.W, H2 = 2LL * g.H, D2 = 2LL * g.D;
    for (; lr < BM; lr += LSTEP) {
      if (mt0 + lr >= g.M) break;
      V8<T> o;
      o.load(El + lr * EPT + cg * 8);
      const long long child = (((long long)n * D2 + 2 * z + tz) * H2 + 2 * y + ty) * W2 + 2 * x + tx;
      o.store(O + child * g.ldo + co);
      x += LSTEP;
      while (x >= g.W) {
        x -= g.W;
        if (++y == g.H) {
          y = 0;
          if (++z == g.D) {
            z = 0;
            ++n;
          }
        }
      }
    }
    return;
  }
  for (int e = threadIdx.x; e < BM * CG; e += 256) {
    const int lr = e / CG, cg = e % CG;
    const long long row = mt0 + lr;
    const int col = nt0 + cg * 8;
    if (row >= g.M || col >= g.Ncols) continue;
    V8<T> o;
    o.load(El + lr * EPT + cg * 8);
    if (MODE == MODE_POINT && g.res) {
      V8<T> rv;
      rv.load(reinterpret_cast<const T*>(g.res) + row * g.ldres + col);
#pragma unroll
      for (int j = 0; j < 8; ++j) o.set(j, o.get(j) + rv.get(j));
    }
    if (MODE == MODE_POINT && g.epi == 1) {
      V8<T> gv;
#pragma unroll
      for (int j = 0; j < 8; ++j) gv.set(j, mmseg_gelu(o.get(j)));
      gv.store(reinterpret_cast<T*>(g.aux_out) + row * g.ldo + col);
    } else if (MODE == MODE_POINT && g.epi == 2) {
      V8<T> hv;
      hv.load(reinterpret_cast<const T*>(g.aux) + row * g.ldo + col);
#pragma unroll
      for (int j = 0; j < 8; ++j) o.set(j, o.get(j) * mmseg_gelu_grad(hv.get(j)));
    }
    o.store(out_at<T>(g, row, col));
  }
}

// ------------------------------------------------------ brick conv (3^3)
// LDS-staged halo tiles for the 3x3x3 convolution (fwd, and dgrad with the
// flipped / transposed weights): a block owns a 4x4x8 output brick (128
// voxels, one sample) x BN output channels.  Per 32-channel input chunk the
// 6x6x10 input halo is staged ONCE into LDS and reused by all 27 taps (the
// per-lane gather kernel above re-reads it 27x through L1/L2), and the chunk's
// weights are staged one kz-plane (9 taps) at a time.  Register prefetch of
// the next stage overlaps its global loads with the current MFMAs.
// Wave w computes brick z-slice w (32 voxels = 2 row tiles) x BN columns.
constexpr int BRK_Z = 4, BRK_Y = 4, BRK_X = 8;
constexpr int HLO_Z = BRK_Z + 2, HLO_Y = BRK_Y + 2, HLO_X = BRK_X + 2;
constexpr int HLO_V = HLO_Z * HLO_Y * HLO_X;   // 360 halo voxels
constexpr int CK = 32;                          // input channels per chunk

template <typename T, int BN>
__global__ __launch_bounds__(256) void conv3_brick_kernel(GemmArgs g) {
  constexpr int EP = 16 / sizeof(T);
  constexpr int XP = CK + EP;                   // halo row pitch (elements)
  constexpr int WP = CK;                        // weight row pitch (elements)
  constexpr int RN = BN / 16;
  constexpr int XS = HLO_V * XP, WS = 9 * BN * WP;
  __shared__ __attribute__((aligned(16))) T lds[XS + WS];
  T* Xl = lds;
  T* Wl = lds + XS;
  constexpr int X_ITEMS = HLO_V * (CK / 8);     // V8 loads per halo stage
  constexpr int X_PER = (X_ITEMS + 255) / 256;
  constexpr int W_ITEMS = 9 * BN * (CK / 8);
  constexpr int W_PER = (W_ITEMS + 255) / 256;

  const T* A = reinterpret_cast<const T*>(g.a);
  const T* Bw = reinterpret_cast<const T*>(g.b);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bz_n = g.D / BRK_Z, by_n = g.H / BRK_Y, bx_n = g.W / BRK_X;
  const int nbrick = (g.M / (g.D * g.H * g.W)) * bz_n * by_n * bx_n;
  const int nt_n = (g.Ncols + BN - 1) / BN;
  const int tile = g.swz ? xcd_swizzle(blockIdx.x, nbrick * nt_n) : (int)blockIdx.x;
  int bidx = tile % nbrick;
  const int nt = tile / nbrick;
  const int bx = bidx % bx_n; bidx /= bx_n;
  const int by = bidx % by_n; bidx /= by_n;
  const int bz = bidx % bz_n;
  const int n = bidx / bz_n;
  const int z0 = bz * BRK_Z, y0 = by * BRK_Y, x0 = bx * BRK_X;
  const long long HW = (long long)g.H * g.W;
  const long long nbase = (long long)n * g.D * HW;
  const int n0 = nt * BN;
  const int cin = 8 << g.cpg_shift;             // channels of the A source
  const int nchunk = gemm_nchunk(g);
  const int nstage = nchunk * 3;

  V8<T> xr[X_PER], wr[W_PER];
  auto load_x = [&](int c) {
#pragma unroll
    for (int k = 0; k < X_PER; ++k) {
      const int e = tid + k * 256;
      if (e < X_ITEMS) {
        const int h = e >> 2, cg = e & 3;
        const int hx = h % HLO_X, hy = (h / HLO_X) % HLO_Y, hz = h / (HLO_X * HLO_Y);
        const int z = z0 - 1 + hz, y = y0 - 1 + hy, x = x0 - 1 + hx;
        if ((unsigned)z < (unsigned)g.D && (unsigned)y < (unsigned)g.H && (unsigned)x < (unsigned)g.W)
          xr[k].load(A + (nbase + z * HW + (long long)y * g.W + x) * g.lda + c * CK + cg * 8);
        else
          xr[k].zero();
      }
    }
  };
  auto load_w = [&](int c, int kz) {
#pragma unroll
    for (int k = 0; k < W_PER; ++k) {
      const int e = tid + k * 256;
      if (e < W_ITEMS) {
        const int cg = e & 3, q = e >> 2;
        const int col = q % BN, t9 = q / BN;
        const int tap = kz * 9 + t9;
        const int kgi = tap * (cin / 8) + c * 4 + cg;
        wr[k].load(Bw + ((long long)kgi * g.Cpad + n0 + col) * 8);
      }
    }
  };
  auto store_x = [&]() {
#pragma unroll
    for (int k = 0; k < X_PER; ++k) {
      const int e = tid + k * 256;
      if (e < X_ITEMS) xr[k].store(Xl + (e >> 2) * XP + (e & 3) * 8);
    }
  };
  auto store_w = [&]() {
#pragma unroll
    for (int k = 0; k < W_PER; ++k) {
      const int e = tid + k * 256;
      if (e < W_ITEMS) {
        const int cg = e & 3, q = e >> 2;   // q = t9*BN + col
        wr[k].store(Wl + q * WP + cg * 8);
      }
    }
  };

  f32x4 acc[2][RN];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // lane's rows: row r = lane&15 of tile i -> brick voxel (wave, 2i + (r>>3), r&7)
  const int r16 = lane & 15, kg = lane >> 4;
  int hrow[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) hrow[i] = (wave * HLO_Y + (2 * i + (r16 >> 3))) * HLO_X + (r16 & 7);

  load_x(0);
  load_w(0, 0);
  store_x();
  store_w();
  __syncthreads();
  for (int st = 0; st < nstage; ++st) {
    const int c = st / 3, kz = st - c * 3;
    const int sn = st + 1;
    const bool more = sn < nstage;
    const int cn = sn / 3, kzn = sn - cn * 3;
    if (more) {
      load_w(cn, kzn);
      if (kzn == 0) load_x(cn);
    }
#pragma unroll
    for (int t9 = 0; t9 < 9; ++t9) {
      const int ky = t9 / 3, kx = t9 - ky * 3;
      const int hoff = (kz * HLO_Y + ky) * HLO_X + kx;
      V8<T> af[2], bf[RN];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i].load(Xl + (hrow[i] + hoff) * XP + kg * 8);
#pragma unroll
      for (int j = 0; j < RN; ++j) bf[j].load(Wl + (t9 * BN + j * 16 + r16) * WP + kg * 8);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j) mfma_step<T>(acc[i][j], af[i], bf[j]);
    }
    __syncthreads();
    if (more) {
      store_w();
      if (kzn == 0) store_x();
      __syncthreads();
    }
  }

  T* O = reinterpret_cast<T*>(g.out);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      const int col = n0 + j * 16 + r16;
      if (col >= g.Ncols) continue;
      const float bv = g.bias ? g.bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = kg * 4 + r;            // 0..15 within the tile
        const int y = y0 + 2 * i + (row >> 3), x = x0 + (row & 7), z = z0 + wave;
        const long long vox = nbase + z * HW + (long long)y * g.W + x;
        *out_at<T>(g, vox, col) = from_f<T>(acc[i][j][r] + bv);
      }
    }
}

// ------------------------------------------------- brick conv v2 (3^3)
// Same algorithm as conv3_brick_kernel with a 2x larger per-wave tile and
// bank-conflict-free LDS images:
//   * block = (4*ZW) x 8 x 8 output voxels x BN columns; wave w owns z-slices
//     [w*ZW, (w+1)*ZW) = 4*ZW row tiles of 16 voxels (two 8-voxel x-rows each),
//     so one B fragment feeds 4*ZW MFMAs and one A fragment feeds BN/16;
//   * halo image: 32 channels of a voxel = 4 consecutive 16-B quads, y-rows
//     padded to 42 quads.  A ds_read_b128 lane group then touches 16 distinct
//     bank quads for every tap shift (checked exhaustively on the host for
//     the lane groups of MI355X_MICROARCH.md §LDS);
//   * weight image: rows of 4 quads, quad index XOR-swizzled by bit 3 of the
//     column, which makes the 16-lane groups conflict-free as well;
//   * epilogue staged through LDS so every lane stores 16-B vectors.
constexpr int B2_Y = 8, B2_X = 8;
constexpr int H2_Y = B2_Y + 2, H2_X = B2_X + 2;

template <typename T>
struct Brick2Layout {
  static constexpr int QV = 2 * (int)sizeof(T);      // 16-B quads per voxel (32 channels): 4 bf16, 8 f32
  static constexpr int QG = QV / 4;                    // quads per 8-channel group
  static constexpr int RY = H2_X * QV + 2;             // quads per halo y-row (padded)
  static constexpr int RZ = H2_Y * RY;                 // quads per halo z-plane
};

__device__ __forceinline__ int w2_swz(int col) { return ((col >> 3) & 1) << 1; }

template <typename T>
__device__ __forceinline__ void buf_load_v8(V8<T>& v, __amdgpu_buffer_rsrc_t r, uint32_t off);

// B32: the halo is staged with 32-bit offset buffer loads whose out-of-volume lanes read zeros (host: the A tensor
// spans < 2^31 bytes), instead of 64-bit address arithmetic and a bounds branch per item.
template <typename T, int BN, int ZW, bool PF = false, bool B32 = false>
__global__ __launch_bounds__(256, sizeof(T) == 2 ? 2 : 1) void conv3_brick2_kernel(GemmArgs g) {
  PROBE_BLOCK(false);
  PROBE_DECL();
  using L = Brick2Layout<T>;
  constexpr int BZ = 4 * ZW, HZ = BZ + 2;
  constexpr int RM = 4 * ZW, RN = BN / 16;
  constexpr int XQ = HZ * L::RZ;                      // halo quads
  constexpr int WQ = 9 * BN * L::QV;                  // weight quads (one kz plane)
  constexpr int EQ = (BZ * 64 * BN * (int)sizeof(T) + 15) / 16;   // epilogue tile quads
  constexpr int LQ = (XQ + WQ) > EQ ? (XQ + WQ) : EQ;
  __shared__ __attribute__((aligned(16))) float4 lds4[LQ];
  T* Xl = reinterpret_cast<T*>(lds4);
  T* Wl = reinterpret_cast<T*>(lds4 + XQ);
  constexpr int EPQ = 16 / sizeof(T);                 // elements per quad
  constexpr int HV = HZ * H2_Y * H2_X;
  constexpr int X_ITEMS = HV * 4;                     // 8-channel groups per halo stage
  constexpr int X_PER = (X_ITEMS + 255) / 256;
  constexpr int W_ITEMS = 9 * BN * 4;
  constexpr int W_PER = (W_ITEMS + 255) / 256;

  const T* A = reinterpret_cast<const T*>(g.a);
  const T* Bw = reinterpret_cast<const T*>(g.b);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bz_n = g.D / BZ, by_n = g.H / B2_Y, bx_n = g.W / B2_X;
  const int nbrick = (g.M / (g.D * g.H * g.W)) * bz_n * by_n * bx_n;
  const int nt_n = (g.Ncols + BN - 1) / BN;
  const int tile = g.swz ? xcd_swizzle(blockIdx.x, nbrick * nt_n) : (int)blockIdx.x;
  int bidx = tile % nbrick;
  const int nt = tile / nbrick;
  const int bx = bidx % bx_n; bidx /= bx_n;
  const int by = bidx % by_n; bidx /= by_n;
  const int bz = bidx % bz_n;
  const int n = bidx / bz_n;
  const int z0 = bz * BZ, y0 = by * B2_Y, x0 = bx * B2_X;
  const long long HW = (long long)g.H * g.W;
  const long long nbase = (long long)n * g.D * HW;
  const int n0 = nt * BN;
  const int cin = 8 << g.cpg_shift;
  const int nchunk = gemm_nchunk(g);
  const int nstage = nchunk * 3;

  V8<T> xr[X_PER], wr[W_PER];
  const int nvox = n * g.D * g.H * g.W;   // (B32 only: the host checked the extent)
  const __amdgpu_buffer_rsrc_t arsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(g.a), 0, B32 ? (int)((long long)g.M * g.lda * (int)sizeof(T)) : 0, 0x00020000);
  auto load_x = [&](int c) {
#pragma unroll
    for (int k = 0; k < X_PER; ++k) {
      const int e = tid + k * 256;
      if (e < X_ITEMS) {
        const int h = e >> 2, cg = e & 3;
        const int hx = h % H2_X, hy = (h / H2_X) % H2_Y, hz = h / (H2_X * H2_Y);
        const int z = z0 - 1 + hz, y = y0 - 1 + hy, x = x0 - 1 + hx;
        const bool ok = (unsigned)z < (unsigned)g.D && (unsigned)y < (unsigned)g.H && (unsigned)x < (unsigned)g.W;
        if constexpr (B32) {
          const uint32_t off = ok ? (uint32_t)(((nvox + (z * g.H + y) * g.W + x) * g.lda + c * CK + cg * 8) *
                                               (int)sizeof(T))
                                  : 0x80000000u;
          buf_load_v8<T>(xr[k], arsrc, off);   // out-of-volume lanes read zeros
        } else {
          if (ok)
            xr[k].load(A + (nbase + z * HW + (long long)y * g.W + x) * g.lda + c * CK + cg * 8);
          else
            xr[k].zero();
        }
      }
    }
  };
  auto store_x = [&]() {
#pragma unroll
    for (int k = 0; k < X_PER; ++k) {
      const int e = tid + k * 256;
      if (e < X_ITEMS) {
        const int h = e >> 2, cg = e & 3;
        const int hx = h % H2_X, hy = (h / H2_X) % H2_Y, hz = h / (H2_X * H2_Y);
        xr[k].store(Xl + (hz * L::RZ + hy * L::RY + hx * L::QV + cg * L::QG) * EPQ);
      }
    }
  };
  auto load_w = [&](int c, int kz) {
#pragma unroll
    for (int k = 0; k < W_PER; ++k) {
      const int e = tid + k * 256;
      if (e < W_ITEMS) {
        const int cg = e & 3, q = e >> 2;
        const int col = q % BN, t9 = q / BN;
        const int kgi = (kz * 9 + t9) * (cin / 8) + c * 4 + cg;
        wr[k].load(Bw + ((long long)kgi * g.Cpad + n0 + col) * 8);
      }
    }
  };
  auto store_w = [&]() {
#pragma unroll
    for (int k = 0; k < W_PER; ++k) {
      const int e = tid + k * 256;
      if (e < W_ITEMS) {
        const int cg = e & 3, q = e >> 2;     // q = t9*BN + col
        wr[k].store(Wl + (q * L::QV + (cg ^ w2_swz(q)) * L::QG) * EPQ);
      }
    }
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int r16 = lane & 15, kg = lane >> 4;
  int aq[RM];   // halo quad of the lane's row for tap (0,0,0), group kg
#pragma unroll
  for (int i = 0; i < RM; ++i) {
    const int zs = wave * ZW + (i >> 2), yr = 2 * (i & 3) + (r16 >> 3), xr_ = r16 & 7;
    aq[i] = zs * L::RZ + yr * L::RY + xr_ * L::QV + kg * L::QG;
  }
  int bq[RN];
#pragma unroll
  for (int j = 0; j < RN; ++j) {
    const int col = j * 16 + r16;
    bq[j] = col * L::QV + (kg ^ w2_swz(col)) * L::QG;
  }

  PROBE_T();
  load_x(0);
  load_w(0, 0);
  store_x();
  store_w();
  __syncthreads();
  PROBE_T();
  for (int st = 0; st < nstage; ++st) {
    const int c = st / 3, kz = st - c * 3;
    const int sn = st + 1;
    const bool more = sn < nstage;
    const int cn = sn / 3, kzn = sn - cn * 3;
    if (more) {
      load_w(cn, kzn);
      if (kzn == 0) load_x(cn);
    }
    if constexpr (PF) {
      // fragments of tap t+1 are read while tap t's MFMAs run (one wave per SIMD cannot hide the LDS latency
      // behind another wave's MFMAs)
      V8<T> af[2][RM], bf[2][RN];
      auto rd = [&](int t9, int b) {
        const int ky = t9 / 3, kx = t9 - ky * 3;
        const int hoff = kz * L::RZ + ky * L::RY + kx * L::QV;
#pragma unroll
        for (int j = 0; j < RN; ++j) bf[b][j].load(Wl + (t9 * BN * L::QV + bq[j]) * EPQ);
#pragma unroll
        for (int i = 0; i < RM; ++i) af[b][i].load(Xl + (aq[i] + hoff) * EPQ);
      };
      rd(0, 0);
#pragma unroll
      for (int t9 = 0; t9 < 9; ++t9) {
        if (t9 < 8) rd(t9 + 1, (t9 + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j) mfma_step<T>(acc[i][j], af[t9 & 1][i], bf[t9 & 1][j]);
      }
    } else {
#pragma unroll
      for (int t9 = 0; t9 < 9; ++t9) {
        const int ky = t9 / 3, kx = t9 - ky * 3;
        const int hoff = kz * L::RZ + ky * L::RY + kx * L::QV;
        V8<T> af[RM], bf[RN];
#pragma unroll
        for (int j = 0; j < RN; ++j) bf[j].load(Wl + (t9 * BN * L::QV + bq[j]) * EPQ);
#pragma unroll
        for (int i = 0; i < RM; ++i) af[i].load(Xl + (aq[i] + hoff) * EPQ);
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j) mfma_step<T>(acc[i][j], af[i], bf[j]);
      }
    }
    PROBE_T();
    __syncthreads();
    if (more) {
      store_w();
      if (kzn == 0) store_x();
      __syncthreads();
    }
    PROBE_T();
  }

  // epilogue: acc (+bias) -> LDS tile [BZ*64 voxels][BN] -> 16-B vector stores
  T* El = reinterpret_cast<T*>(lds4);
  constexpr int EP = BN + 8;   // padded pitch (elements)
  static_assert(BZ * 64 * (BN + 8) * sizeof(T) + 2048 <= LQ * 16, "epilogue tile (+ stats scratch) must fit");
#pragma unroll
  for (int j = 0; j < RN; ++j) {
    const int col = j * 16 + r16;
    const float bv = (g.bias && n0 + col < g.Ncols) ? g.bias[n0 + col] : 0.f;
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int v = (wave * ZW + (i >> 2)) * 64 + (2 * (i & 3)) * 8 + kg * 4 + r;   // voxel in brick (z,y,x)
        El[v * EP + col] = from_f<T>(acc[i][j][r] + bv);
      }
  }
  __syncthreads();
  if (g.stats) {
    float* red = reinterpret_cast<float*>(El + BZ * 64 * EP);
    const long long brick = (long long)n * (bz_n * by_n * bx_n) + ((long long)bz * by_n + by) * bx_n + bx;
    brick_in_stats<T, BN>(El, EP, BZ * 64, red, g.stats, brick, n0, g.Ncols);
  }
  T* O = reinterpret_cast<T*>(g.out);
  constexpr int CG = BN / 8;                  // 8-column groups per voxel
  constexpr int O_ITEMS = BZ * 64 * CG;
  // zero groups past Ncols (whole-row hint), written by the last column tile's first groups
  const int zg = (g.zcols > g.Ncols && n0 + BN >= g.Ncols) ? (g.zcols - g.Ncols) >> 3 : 0;
#pragma unroll
  for (int k = 0; k < O_ITEMS / 256; ++k) {
    const int e = tid + k * 256;
    const int v = e / CG, cg = e % CG;
    const int col = n0 + cg * 8;
    const int z = z0 + (v >> 6), y = y0 + ((v >> 3) & 7), x = x0 + (v & 7);
    if (col < g.Ncols) {
      V8<T> o;
      o.load(El + v * EP + cg * 8);
      o.store(out_at<T>(g, nbase + z * HW + (long long)y * g.W + x, col));
    }
    for (int zc = cg; zc < zg; zc += CG) {
      V8<T> zv;
      zv.zero();
      zv.store(O + (nbase + z * HW + (long long)y * g.W + x) * g.ldo + g.Ncols + zc * 8);
    }
  }
  PROBE_T();
  PROBE_BLOCK(true);
}


// ------------------------------------------------- brick conv v3 (3^3)
// conv3_brick2_kernel (same 4x8x8-voxel brick, halo / weight LDS images and
// 9-tap stages) with the per-block fixed costs cut, which at Cin = 32 (one
// chunk, three stages per block) were ~5 VALU per MFMA (rocprofv3
// SQ_INSTS_VALU / SQ_INSTS_MFMA on the 96^3 layers):
//   * halo staging: thread t < 240 owns one (x, 8-channel group) column of the
//     halo and walks its 60 (z, y) rows 6 apart, so the voxel offset, the LDS
//     slot and the z / y bounds advance by block-uniform steps; the loads are
//     buffer loads whose out-of-volume lanes carry an offset past the buffer
//     end and read zeros (no branch, no zero fill);
//   * the MFMA computes the transposed tile W^T X (A and B swapped), so a lane
//     holds 4 consecutive output channels of one voxel: bias, bf16 packing and
//     an 8-B global store straight from the accumulators, no LDS epilogue.
template <typename T>
__device__ __forceinline__ void buf_load_v8(V8<T>& v, __amdgpu_buffer_rsrc_t r, uint32_t off);
template <>
__device__ __forceinline__ void buf_load_v8<bf16_t>(V8<bf16_t>& v, __amdgpu_buffer_rsrc_t r, uint32_t off) {
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  const i32x4 t = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  v.v = __builtin_bit_cast(bf16x8, t);
}
// The whole vector is bit-cast at once.  Casting element by element (__builtin_bit_cast(float, a[j])) is
// miscompiled by hipcc (ROCm 7.2, gfx950): the b128 loads were narrowed to buffer_load_dword and element 0 was
// copied into all four registers (v173..v175 = v172 in the disassembly), which is why the fp32 instantiation
// of the 32-bit staging gave wrong results in r02 (tests/test_kernels_gpu.py::test_b32_halo_staging).
template <>
__device__ __forceinline__ void buf_load_v8<float>(V8<float>& v, __amdgpu_buffer_rsrc_t r, uint32_t off) {
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  const f32x4v a = __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
  const f32x4v b = __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(r, off + 16, 0, 0));
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v.v[j] = a[j];
    v.v[4 + j] = b[j];
  }
}

// Measured and removed (round 6 knob pruning; numbers in DESIGN): a double-buffered weight stage (1 % slower),
// the next halo chunk loaded at the first stage of the current one (4 % slower on the bench), unconditional
// clamped weight loads, and sched_group_barrier interleaving of the fragment reads (8-13 % slower).
template <typename T, int BN>
__global__ __launch_bounds__(256, sizeof(T) == 2 ? 2 : 1) void conv3_brick3_kernel(GemmArgs g, int upb) {
  using L = Brick2Layout<T>;
  constexpr int BZ = 4, HZ = BZ + 2;
  constexpr int RM = 4, RN = BN / 16;
  constexpr int XQ = HZ * L::RZ;
  constexpr int WQ = 9 * BN * L::QV;
  __shared__ __attribute__((aligned(16))) float4 lds4[XQ + WQ];
  T* Xl = reinterpret_cast<T*>(lds4);
  T* Wl = reinterpret_cast<T*>(lds4 + XQ);
  constexpr int EPQ = 16 / sizeof(T);
  constexpr int XROWS = HZ * H2_Y;                    // 60 (z, y) halo rows
  constexpr int XK = XROWS / 6;                       // rows per thread (6 rows per pass of 240 threads)
  constexpr int W_ITEMS = 9 * BN * 4;
  constexpr int W_PER = (W_ITEMS + 255) / 256;
  static_assert(XROWS % 6 == 0, "halo rows per pass");

  const T* Bw = reinterpret_cast<const T*>(g.b);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bz_n = g.D / BZ, by_n = g.H / B2_Y, bx_n = g.W / B2_X;
  const int nbrick = (g.M / (g.D * g.H * g.W)) * bz_n * by_n * bx_n;
  const int nt_n = (g.Ncols + BN - 1) / BN;
  const int units = nbrick * nt_n;
  // this block's units: a contiguous range (consecutive units share halo columns in L2); unit = brick * nt_n + nt
  const int blk = g.swz ? xcd_swizzle(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int u_begin = blk * upb;
  const int u_end = u_begin + upb < units ? u_begin + upb : units;
  if (u_begin >= u_end) return;
  const int HW = g.H * g.W;
  const int cin = 8 << g.cpg_shift;
  const int nchunk = gemm_nchunk(g);
  const int nstage = nchunk * 3;
  const int ldb = g.lda * (int)sizeof(T);            // bytes per voxel
  const int vox_per_n = g.D * HW;

  // ---- halo column of this thread: (hx, cg) fixed, rows r0, r0+6, ... (hz = r / 10, hy = r % 10)
  const __amdgpu_buffer_rsrc_t arsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(g.a), 0, (int)((long long)(g.M / vox_per_n) * vox_per_n * ldb), 0x00020000);
  const bool xact = tid < 240;
  const int xq = tid % 40, r0 = tid / 40;
  const int hx = xq >> 2, cg = xq & 3;
  // row r0 + 6k -> (hz, hy) = divmod by 10 ((row * 205) >> 11 is exact for row < 1029); recomputed where
  // used rather than kept in 2 x XK registers (the BN64 instantiation is at the 256-VGPR cap)
  auto row_hz = [&](int k) { return ((r0 + 6 * k) * 205) >> 11; };
  const int xlds0 = (hx * L::QV + cg * L::QG) * EPQ;
  struct Unit { int n, z0, y0, x0, n0; };
  auto unit_of = [&](int u) {
    Unit r;
    const int nt = u % nt_n;
    int b = u / nt_n;
    const int bx = b % bx_n; b /= bx_n;
    const int by = b % by_n; b /= by_n;
    r.z0 = (b % bz_n) * BZ;
    r.n = b / bz_n;
    r.y0 = by * B2_Y;
    r.x0 = bx * B2_X;
    r.n0 = nt * BN;
    return r;
  };
  uint32_t xoff[XK];
  auto set_x = [&](const Unit& q) {    // per-unit halo offsets; out-of-volume lanes point past the buffer end
    const int xx = q.x0 - 1 + hx;
    const bool xok = xact && (unsigned)xx < (unsigned)g.W;
    const int vb = q.n * vox_per_n + xx;
#pragma unroll
    for (int k = 0; k < XK; ++k) {
      const int hz = row_hz(k), hy = r0 + 6 * k - 10 * hz;
      const int zz = q.z0 - 1 + hz, yy = q.y0 - 1 + hy;
      const bool ok = xok && (unsigned)zz < (unsigned)g.D && (unsigned)yy < (unsigned)g.H;
      xoff[k] = ok ? (uint32_t)((vb + zz * HW + yy * g.W) * ldb + cg * 8 * (int)sizeof(T)) : 0x80000000u;
    }
  };
  V8<T> xr[XK], wr[W_PER];
  auto load_x = [&](int c) {
    const uint32_t coff = (uint32_t)(c * CK * (int)sizeof(T));
#pragma unroll
    for (int k = 0; k < XK; ++k) buf_load_v8<T>(xr[k], arsrc, xoff[k] + coff);   // OOB lanes read 0
  };
  auto store_x = [&]() {
    if (xact) {
#pragma unroll
      for (int k = 0; k < XK; ++k) {
        const int hz = row_hz(k), hy = r0 + 6 * k - 10 * hz;
        xr[k].store(Xl + xlds0 + (hz * L::RZ + hy * L::RY) * EPQ);
      }
    }
  };
  // Every thread issues W_PER loads / stores unconditionally (items past the stage are clamped onto the
  // last item: a duplicate load and an identical store), so the compiler cannot sink a predicated load
  // past the tap loop, where its latency would be exposed right before store_w.
  auto load_w = [&](int n0, int c, int kz) {
#pragma unroll
    for (int k = 0; k < W_PER; ++k) {
      const int e0 = tid + k * 256;
      if (e0 < W_ITEMS) {
        const int e = e0;
        const int cgw = e & 3, q = e >> 2;
        const int col = q % BN, t9 = q / BN;
        const int kgi = (kz * 9 + t9) * (cin / 8) + c * 4 + cgw;
        wr[k].load(Bw + ((long long)kgi * g.Cpad + n0 + col) * 8);
      }
    }
  };
  auto store_w = [&]() {
    T* Wd = Wl;
#pragma unroll
    for (int k = 0; k < W_PER; ++k) {
      const int e0 = tid + k * 256;
      if (e0 < W_ITEMS) {
        const int e = e0;
        const int cgw = e & 3, q = e >> 2;
        wr[k].store(Wd + (q * L::QV + (cgw ^ w2_swz(q)) * L::QG) * EPQ);
      }
    }
  };

  const int r16 = lane & 15, kg = lane >> 4;
  int aq[RM];
#pragma unroll
  for (int i = 0; i < RM; ++i) {
    const int yr = 2 * (i & 3) + (r16 >> 3), xr_ = r16 & 7;
    aq[i] = wave * L::RZ + yr * L::RY + xr_ * L::QV + kg * L::QG;
  }
  int bq[RN];
#pragma unroll
  for (int j = 0; j < RN; ++j) {
    const int col = j * 16 + r16;
    bq[j] = col * L::QV + (kg ^ w2_swz(col)) * L::QG;
  }
  T* O = reinterpret_cast<T*>(g.out);

  Unit cur = unit_of(u_begin);
  set_x(cur);
  load_x(0);
  load_w(cur.n0, 0, 0);
  store_x();
  store_w();
  __syncthreads();
  for (int u = u_begin; u < u_end; ++u) {
    f32x4 acc[RM][RN];
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const bool unext = u + 1 < u_end;
    Unit nxt = cur;
    if (unext) nxt = unit_of(u + 1);
    for (int st = 0; st < nstage; ++st) {
      const int c = st / 3, kz = st - c * 3;
      // next stage: (cn, kzn) of this unit, or stage 0 of the next unit
      const bool last = st + 1 == nstage;
      const bool more = !last || unext;
      const int sn = last ? 0 : st + 1;
      const int cn = sn / 3, kzn = sn - cn * 3;
      if (more) {
        if (last) set_x(nxt);
        load_w(last ? nxt.n0 : cur.n0, cn, kzn);
        if (kzn == 0) load_x(cn);
      }
#pragma unroll
      for (int t9 = 0; t9 < 9; ++t9) {
        const int ky = t9 / 3, kx = t9 - ky * 3;
        const int hoff = kz * L::RZ + ky * L::RY + kx * L::QV;
        V8<T> af[RM], bf[RN];
#pragma unroll
        for (int j = 0; j < RN; ++j) bf[j].load(Wl + (t9 * BN * L::QV + bq[j]) * EPQ);
#pragma unroll
        for (int i = 0; i < RM; ++i) af[i].load(Xl + (aq[i] + hoff) * EPQ);
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j) mfma_step<T>(acc[i][j], bf[j], af[i]);   // transposed: rows = channels
      }
      __syncthreads();
      if (more) {
        store_w();
        if (kzn == 0) store_x();
        __syncthreads();
      }
    }
    // epilogue: lane holds channels n0 + j*16 + 4*kg + (0..3) of voxel r16 of row tile i
    const long long obase = (long long)cur.n * vox_per_n;
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      const int col = cur.n0 + j * 16 + 4 * kg;
      if (col >= g.Ncols) continue;
      float bv[4] = {0.f, 0.f, 0.f, 0.f};
      if (g.bias) {
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[r] = g.bias[col + r];   // the bias view is only 4-B aligned
      }
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        const int z = cur.z0 + wave, y = cur.y0 + 2 * (i & 3) + (r16 >> 3), x = cur.x0 + (r16 & 7);
        T* dst = out_at<T>(g, obase + (long long)(z * g.H + y) * g.W + x, col);
        if constexpr (sizeof(T) == 2) {
          typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
          bf16x4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = (bf16_t)(acc[i][j][r] + bv[r]);
          *reinterpret_cast<bf16x4*>(dst) = o;
        } else {
          *reinterpret_cast<float4*>(dst) = make_float4(acc[i][j][0] + bv[0], acc[i][j][1] + bv[1],
                                                        acc[i][j][2] + bv[2], acc[i][j][3] + bv[3]);
        }
      }
    }
    cur = nxt;
  }
}

// ------------------------------------------------- brick conv v4 (3^3, bf16, Cin = 32, Co tile 32)
// The 96^3 32 -> 32 layers.  v3 restages the 9-tap weight slab of every (brick, kz) stage through LDS and
// every wave re-reads the same B fragments: per tap and wave 4 A + 2 B ds_read_b128 for 8 MFMAs, plus
// 54 KB of weight and 38 KB of halo LDS writes per brick, and two barriers per stage.  v4:
//   * the whole 27-tap x 32-ci x 32-co weight tile of the block's column tile lives in the accumulator
//     register file (27 x 2 fragments = 216 AGPRs, loaded once per block straight from the packed
//     [KG][Cpad][8] image, which is already fragment-ordered; mfma_aw); LDS holds only halos;
//   * one block of 4 waves per CU (1 wave / SIMD), persistent over a contiguous brick range; the halo is
//     double-buffered: the next brick's halo is loaded into registers when a brick starts and written to the
//     other LDS buffer after 15 taps, so one barrier per brick;
//   * each tap's 4 A reads are issued two taps ahead of their MFMAs (sched_barrier; left alone, hipcc
//     issues them just before their MFMAs).
// Measured (s_memtime stamps, 96^3 B=2 forward): ~200 cycles per tap against 128 of MFMA issue, and the
// tap loop speeds up in proportion when the per-tap A reads are cut (half the reads: 146 cycles per tap):
// the LDS read stream, not latency, barriers or the halo loads, is what bounds this kernel.
// Requirements (host): bf16, one 32-channel K chunk, Ncols % 32 == 0, D % 4, H % 8, W % 8, no fused stats.

// MFMA with the weight fragment pinned to the accumulator file: hipcc otherwise keeps the 216 weight
// registers in VGPRs and, short of VGPRs, issues each tap's LDS reads just before their MFMAs.  The asm is one
// opaque instruction to hipcc: it inserts the lgkmcnt waits for x, but no MFMA hazard padding, which
// brick4_fence / brick4_wfence supply where the accumulators are read and after the weights are written.
__device__ __forceinline__ void mfma_aw(f32x4& acc, const bf16x8& w, const bf16x8& x) {
  asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "a"(w), "v"(x));
}
// e4m3 x e4m3 -> f32 (K = 32: a lane holds 8 fp8 = 8 bytes of A and of B, the bf16 form's lane map)
__device__ __forceinline__ void mfma_aw8(f32x4& acc, const long& w, const long& x) {
  asm("v_mfma_f32_16x16x32_fp8_fp8 %0, %1, %2, %0" : "+a"(acc) : "a"(w), "v"(x));
}
__device__ __forceinline__ void mfma_aw80(f32x4& acc, const long& w, const long& x) {
  asm("v_mfma_f32_16x16x32_fp8_fp8 %0, %1, %2, 0" : "=a"(acc) : "a"(w), "v"(x));
}
// first MFMA of an accumulation chain: C = 0 (no accumulator zeroing per brick)
__device__ __forceinline__ void mfma_aw0(f32x4& acc, const bf16x8& w, const bf16x8& x) {
  asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc) : "a"(w), "v"(x));
}
__device__ __forceinline__ void brick4_fence(f32x4& a, f32x4& b) {
  asm volatile("s_nop 7\n\ts_nop 7" : "+a"(a), "+a"(b));
}
__device__ __forceinline__ void brick4_wfence(bf16x8& a, bf16x8& b) {
  asm volatile("s_nop 2" : "+a"(a), "+a"(b));
}

__global__ __launch_bounds__(256, 1) void conv3_brick4_kernel(GemmArgs g, int upb, int blocks_per_nt) {
  using T = bf16_t;
  using L = Brick2Layout<T>;
  constexpr int BZ = 4, HZ = BZ + 2;
  constexpr int RM = 4, RN = 2;
  constexpr int PF = 2;                               // A-fragment prefetch distance (taps)
  constexpr int XQ = HZ * L::RZ;
  __shared__ __attribute__((aligned(16))) float4 lds4[2 * XQ];
  T* Xl = reinterpret_cast<T*>(lds4);
  constexpr int EPQ = 8;
  constexpr int XROWS = HZ * H2_Y;                    // 60 (z, y) halo rows
  constexpr int XK = XROWS / 6;                       // rows per thread (6 rows per pass of 240 threads)

  const T* Bw = reinterpret_cast<const T*>(g.b);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bz_n = g.D / BZ, by_n = g.H / B2_Y, bx_n = g.W / B2_X;
  const int nbrick = (g.M / (g.D * g.H * g.W)) * bz_n * by_n * bx_n;
  const int blk_all = g.swz ? xcd_swizzle(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int nt = blk_all / blocks_per_nt, blk = blk_all - nt * blocks_per_nt;
  const int n0 = nt * 32;
  const int u_begin = blk * upb;
  const int u_end = u_begin + upb < nbrick ? u_begin + upb : nbrick;
  if (u_begin >= u_end || n0 >= g.Ncols) return;
  const int HW = g.H * g.W;
  const int cin = 8 << g.cpg_shift;
  const int ldb = g.lda * (int)sizeof(T);
  const int vox_per_n = g.D * HW;
  const int r16 = lane & 15, kg = lane >> 4;

  // ---- weights: fragment (tap, j) = 8 input channels kg*8.. of output column n0 + j*16 + r16
  V8<T> wf[27][RN];
#pragma unroll
  for (int t = 0; t < 27; ++t)
#pragma unroll
    for (int j = 0; j < RN; ++j)
      wf[t][j].load(Bw + ((long long)(t * (cin / 8) + kg) * g.Cpad + n0 + j * 16 + r16) * 8);
#pragma unroll
  for (int t = 0; t < 27; ++t) brick4_wfence(wf[t][0].v, wf[t][1].v);

  // ---- halo column of this thread: (hx, cg) fixed, rows r0, r0+6, ... (hz = r / 10, hy = r % 10)
  const __amdgpu_buffer_rsrc_t arsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(g.a), 0, (int)((long long)(g.M / vox_per_n) * vox_per_n * ldb), 0x00020000);
  const bool xact = tid < 240;
  const int xq = tid % 40, r0 = tid / 40;
  const int hx = xq >> 2, cg = xq & 3;
  auto row_hz = [&](int k) { return ((r0 + 6 * k) * 205) >> 11; };
  const int xlds0 = (hx * L::QV + cg * L::QG) * EPQ;
  struct Unit { int n, z0, y0, x0; };
  auto unit_of = [&](int b) {
    Unit r;
    const int bx = b % bx_n; b /= bx_n;
    const int by = b % by_n; b /= by_n;
    r.z0 = (b % bz_n) * BZ;
    r.n = b / bz_n;
    r.y0 = by * B2_Y;
    r.x0 = bx * B2_X;
    return r;
  };
  V8<T> xr[XK];
  auto load_x = [&](const Unit& q) {    // out-of-volume lanes point past the buffer end and read zeros
    const int xx = q.x0 - 1 + hx;
    const bool xok = xact && (unsigned)xx < (unsigned)g.W;
    const int vb = q.n * vox_per_n + xx;
#pragma unroll
    for (int k = 0; k < XK; ++k) {
      const int hz = row_hz(k), hy = r0 + 6 * k - 10 * hz;
      const int zz = q.z0 - 1 + hz, yy = q.y0 - 1 + hy;
      const bool ok = xok && (unsigned)zz < (unsigned)g.D && (unsigned)yy < (unsigned)g.H;
      const uint32_t off = ok ? (uint32_t)((vb + zz * HW + yy * g.W) * ldb + cg * 16) : 0x80000000u;
      buf_load_v8<T>(xr[k], arsrc, off);
    }
  };
  auto store_x = [&](int buf) {
    if (xact) {
#pragma unroll
      for (int k = 0; k < XK; ++k) {
        const int hz = row_hz(k), hy = r0 + 6 * k - 10 * hz;
        xr[k].store(Xl + buf * XQ * EPQ + xlds0 + (hz * L::RZ + hy * L::RY) * EPQ);
      }
    }
  };
  int aq[RM];
#pragma unroll
  for (int i = 0; i < RM; ++i) {
    const int yr = 2 * i + (r16 >> 3), xr_ = r16 & 7;
    aq[i] = wave * L::RZ + yr * L::RY + xr_ * L::QV + kg * L::QG;
  }
  float bv[RN][4];
#pragma unroll
  for (int j = 0; j < RN; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[j][r] = g.bias ? g.bias[n0 + j * 16 + 4 * kg + r] : 0.f;
  T* O = reinterpret_cast<T*>(g.out);

  Unit cur = unit_of(u_begin);
  load_x(cur);
  store_x(0);
  __syncthreads();
  int b = 0;
  // (Storing each brick's outputs a few taps into the next brick, from a second accumulator set, measured
  // 25 % slower; loading the next halo in two halves, or storing it later, measured no faster.)
  for (int u = u_begin; u < u_end; ++u) {
    f32x4 acc[RM][RN];
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const bool unext = u + 1 < u_end;
    Unit nxt = cur;
    if (unext) {
      nxt = unit_of(u + 1);
      load_x(nxt);
    }
    const T* Xb = Xl + b * XQ * EPQ;
    auto hoff = [](int t) { return (t / 9) * L::RZ + ((t / 3) % 3) * L::RY + (t % 3) * L::QV; };
    V8<T> af[PF + 1][RM];
#pragma unroll
    for (int p = 0; p < PF; ++p)
#pragma unroll
      for (int i = 0; i < RM; ++i) af[p][i].load(Xb + (aq[i] + hoff(p)) * EPQ);
#pragma unroll
    for (int t = 0; t < 27; ++t) {
      if (t == 15 && unext) store_x(b ^ 1);
      if (t + PF < 27) {
#pragma unroll
        for (int i = 0; i < RM; ++i) af[(t + PF) % (PF + 1)][i].load(Xb + (aq[i] + hoff(t + PF)) * EPQ);
      }
      __builtin_amdgcn_sched_barrier(0);   // keep the reads PF taps ahead of their MFMAs
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j) mfma_aw(acc[i][j], wf[t][j].v, af[t % (PF + 1)][i].v);   // rows = channels
    }
#pragma unroll
    for (int i = 0; i < RM; ++i) brick4_fence(acc[i][0], acc[i][1]);
    // epilogue: lane holds channels n0 + j*16 + 4*kg + (0..3) of voxel r16 of row tile i
    const long long obase = (long long)cur.n * vox_per_n;
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      const int col = n0 + j * 16 + 4 * kg;
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        const int z = cur.z0 + wave, y = cur.y0 + 2 * i + (r16 >> 3), x = cur.x0 + (r16 & 7);
        T* dst = out_at<T>(g, obase + (long long)(z * g.H + y) * g.W + x, col);
        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (bf16_t)(acc[i][j][r] + bv[j][r]);
        *reinterpret_cast<bf16x4*>(dst) = o;
      }
    }
    __syncthreads();   // buffer b^1 is complete; buffer b is free for the brick after next
    b ^= 1;
    cur = nxt;
  }
}

// ------------------------------------------------- brick conv v5 (3^3, bf16, Cin = 32, Co tile 32)
// brick4 with the A-read stream halved.  A row tile is 16 consecutive x voxels of ONE y row (brick 4 z x
// 4 y x 16 x, one z plane per wave), so the fragment of row tile i at tap ky is the fragment of halo row
// i + ky: per (kz, kx) the 12 (ky, i) fragments are 6 distinct halo rows, read once and used by 24 MFMAs
// (0.25 ds_read_b128 per MFMA instead of 0.5).  Halo image: voxel = 4 quads of 8 channels, the quad of
// channel group kg at slot kg ^ (((hx >> 2) & 1) << 1), which makes the 16-lane groups of ds_read_b128
// conflict-free for all three kx shifts; rows of 18 voxels, no padding.
// Requirements (host): bf16, one 32-channel K chunk, Ncols % 32 == 0, D % 4, H % 4, W % 16, no fused stats.
// INP (with DMA: the halo staging registers are free for it): the epilogue also sums the InstanceNorm-backward
// partials of its output (GemmArgs::inpart); x of the brick is loaded during the brick's MFMA groups 4..5.
template <bool DBG = false, bool DMA = false, bool INP = false>
__global__ __launch_bounds__(256, 1) void conv3_brick5_kernel(GemmArgs g, int upb, int blocks_per_nt,
                                                              long long* dbg = nullptr) {
  using T = bf16_t;
  constexpr int BZ = 4, BY = 4, BX = 16;
  constexpr int HZ = BZ + 2, HY = BY + 2, HX = BX + 2;
  constexpr int RY = HX * 4, RZ = HY * RY;             // quads per halo row / plane
  constexpr int XQ = HZ * RZ;                          // 2592 quads = 41.5 KB
  constexpr int RN = 2;
  constexpr int XROWS = HZ * HY;                       // 36 (z, y) halo rows
  constexpr int XK = XROWS / 3;                        // rows per thread (3 rows per pass of 216 threads)
  __shared__ __attribute__((aligned(16))) float4 lds4[2 * XQ];
  T* Xl = reinterpret_cast<T*>(lds4);
  constexpr int EPQ = 8;

  const T* Bw = reinterpret_cast<const T*>(g.b);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bz_n = g.D / BZ, by_n = g.H / BY, bx_n = g.W / BX;
  const int nbrick = (g.M / (g.D * g.H * g.W)) * bz_n * by_n * bx_n;
  const int blk_all = g.swz ? xcd_swizzle(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int nt = blk_all / blocks_per_nt, blk = blk_all - nt * blocks_per_nt;
  const int n0 = nt * 32;
  const int u_begin = blk * upb;
  const int u_end = u_begin + upb < nbrick ? u_begin + upb : nbrick;
  if (u_begin >= u_end || n0 >= g.Ncols) return;
  const int HW = g.H * g.W;
  const int cin = 8 << g.cpg_shift;
  const int ldb = g.lda * (int)sizeof(T);
  const int vox_per_n = g.D * HW;
  const int r16 = lane & 15, kg = lane >> 4;
  // timing probe (DBG): lane 0 of waves 0 / 3 of blocks 0 and 100 record (s_memtime, s_memrealtime) pairs
  long long* dp = nullptr;
  int dn = 0;
  if constexpr (DBG) {
    const int sl = (blockIdx.x == 0 ? 0 : blockIdx.x == 100 ? 2 : -9) + (tid == 0 ? 0 : tid == 192 ? 1 : -9);
    if (sl >= 0) dp = dbg + sl * 128;
  }
  auto stamp = [&]() {
    if constexpr (DBG) {
      if (dp && dn < 64) {
        dp[64 + dn] = (long long)__builtin_amdgcn_s_memrealtime();
        dp[dn++] = (long long)__builtin_amdgcn_s_memtime();
      }
    }
  };
  stamp();

  V8<T> wf[27][RN];
#pragma unroll
  for (int t = 0; t < 27; ++t)
#pragma unroll
    for (int j = 0; j < RN; ++j)
      wf[t][j].load(Bw + ((long long)(t * (cin / 8) + kg) * g.Cpad + n0 + 8 * (r16 >> 2) + 4 * j + (r16 & 3)) * 8);
#pragma unroll
  for (int t = 0; t < 27; ++t) brick4_wfence(wf[t][0].v, wf[t][1].v);

  // ---- halo staging: thread t < 216 owns quad column (hx, cg) = divmod(t % 72, 4) of rows t / 72 + 3k
  const __amdgpu_buffer_rsrc_t arsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(g.a), 0, (int)((long long)(g.M / vox_per_n) * vox_per_n * ldb), 0x00020000);
  const bool xact = tid < 216;
  const int xq = tid % 72, r0 = tid / 72;
  const int hx = xq >> 2, cg = xq & 3;
  const int xlds0 = (hx * 4 + (cg ^ (((hx >> 2) & 1) << 1))) * EPQ;
  struct Unit { int n, z0, y0, x0; };
  auto unit_of = [&](int b) {
    Unit r;
    const int bx = b % bx_n; b /= bx_n;
    const int by = b % by_n; b /= by_n;
    r.z0 = (b % bz_n) * BZ;
    r.n = b / bz_n;
    r.y0 = by * BY;
    r.x0 = bx * BX;
    return r;
  };
  V8<T> xr[XK];
  // byte offset of row k's element relative to the halo origin (z0 - 1, y0 - 1, x0 - 1), fixed per thread
  uint32_t rel[XK];
#pragma unroll
  for (int k = 0; k < XK; ++k) {
    const int row = r0 + 3 * k, hz = row / HY, hy = row - hz * HY;
    rel[k] = (uint32_t)((hz * HW + hy * g.W + hx) * ldb + cg * 16);
  }
  // halo offsets of a brick: z / y interior bricks need one x test per lane (the unit base is uniform);
  // border bricks test every row.  Out-of-volume lanes point past the buffer end and read zeros.
  uint32_t xo[XK];
  // deferred norm of the A source: the statistics of the sample of the brick being staged (set_x runs once per
  // staged brick, before its store_x)
  float nmu[8], nrs[8];
  int norm_n = -1;
  auto set_x = [&](const Unit& q) {
    if (g.nmean && q.n != norm_n) {
      norm_n = q.n;
      const int cb = q.n * cin + cg * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        nmu[j] = g.nmean[cb + j];
        nrs[j] = g.nrstd[cb + j];
      }
    }
    const int xx = q.x0 - 1 + hx;
    const bool xok = xact && (unsigned)xx < (unsigned)g.W;
    const int ob = ((q.n * g.D + q.z0 - 1) * g.H + q.y0 - 1) * g.W + q.x0 - 1;   // origin voxel (may be -1)
    const uint32_t base = (uint32_t)(ob * ldb);
    if (q.z0 >= 1 && q.z0 + BZ < g.D && q.y0 >= 1 && q.y0 + BY < g.H) {
#pragma unroll
      for (int k = 0; k < XK; ++k) xo[k] = xok ? base + rel[k] : 0x80000000u;
    } else {
#pragma unroll
      for (int k = 0; k < XK; ++k) {
        const int row = r0 + 3 * k, hz = row / HY, hy = row - hz * HY;
        const int zz = q.z0 - 1 + hz, yy = q.y0 - 1 + hy;
        const bool ok = xok && (unsigned)zz < (unsigned)g.D && (unsigned)yy < (unsigned)g.H;
        xo[k] = ok ? base + rel[k] : 0x80000000u;
      }
    }
  };
  auto load_x = [&](int k0, int k1) {
#pragma unroll
    for (int k = k0; k < k1; ++k) buf_load_v8<T>(xr[k], arsrc, xo[k]);
  };
  // DMA: the halo goes straight from HBM into the LDS image (buffer_load ... lds; no staging registers, no
  // ds_write).  Wave-instruction m covers image quads [64 m, 64 m + 64); wave w issues m = w, w + 4, ...
  constexpr int DM = (XQ + 63) / 64;                  // 41 wave-instructions per halo
  constexpr int DK = (DM + 3) / 4;                    // per wave (the last ones partly or wholly empty)
  uint32_t drel[DK];                                  // lane's byte offset from the halo origin, or ~0u (no quad)
  uint32_t dlm = 0, drm = 0;                          // bit k: lane's quad k is in halo column hx = 0 / hx = 17
#pragma unroll
  for (int kk = 0; kk < DK; ++kk) {
    const int p = (wave + 4 * kk) * 64 + lane;
    const int row = p / RY, qi = p - row * RY, h = qi >> 2, sl = qi & 3;
    const int c = sl ^ (((h >> 2) & 1) << 1);
    const int hz = row / HY, hy = row - hz * HY;
    drel[kk] = p < XQ ? (uint32_t)((hz * HW + hy * g.W + h) * ldb + c * 16) : ~0u;
    if (h == 0) dlm |= 1u << kk;
    if (h == HX - 1) drm |= 1u << kk;
  }
  uint32_t dof[DK];
  auto set_xd = [&](const Unit& q) {
    const int ob = ((q.n * g.D + q.z0 - 1) * g.H + q.y0 - 1) * g.W + q.x0 - 1;
    const uint32_t base = (uint32_t)(ob * ldb);
    const uint32_t xbad = (q.x0 == 0 ? dlm : 0u) | (q.x0 + BX == g.W ? drm : 0u);
    const bool inner = q.z0 >= 1 && q.z0 + BZ < g.D && q.y0 >= 1 && q.y0 + BY < g.H;
#pragma unroll
    for (int kk = 0; kk < DK; ++kk) {
      bool ok = drel[kk] != ~0u && !((xbad >> kk) & 1u);
      if (!inner) {
        const int p = (wave + 4 * kk) * 64 + lane;
        const int row = p / RY, hz = row / HY, hy = row - hz * HY;
        ok = ok && (unsigned)(q.z0 - 1 + hz) < (unsigned)g.D && (unsigned)(q.y0 - 1 + hy) < (unsigned)g.H;
      }
      dof[kk] = ok ? base + drel[kk] : 0x80000000u;
    }
  };
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  auto issue_xd = [&](int buf, int k0, int k1) {
#pragma unroll
    for (int kk = k0; kk < k1; ++kk) {
      if (wave + 4 * kk < DM)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            arsrc, (lds_ptr_t)(lds4 + buf * XQ + (wave + 4 * kk) * 64), 16, dof[kk], 0, 0, 0);
    }
  };
  auto store_x = [&](int buf, int k0, int k1) {
    if (xact) {
#pragma unroll
      for (int k = k0; k < k1; ++k) {
        if (g.nmean && xo[k] != 0x80000000u) norm_relu8<T>(xr[k], nmu, nrs);   // padding stays 0
        xr[k].store(Xl + (buf * XQ + (r0 + 3 * k) * RY) * EPQ + xlds0);
      }
    }
  };
  // per-lane A offsets (quads) of the three kx shifts: voxel hx = r16 + kx, channel group kg
  int ao[3];
#pragma unroll
  for (int kx = 0; kx < 3; ++kx) {
    const int h = r16 + kx;
    ao[kx] = wave * RZ + h * 4 + (kg ^ (((h >> 2) & 1) << 1));
  }
  float bv[RN][4];
#pragma unroll
  for (int j = 0; j < RN; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[j][r] = g.bias ? g.bias[n0 + 8 * kg + 4 * j + r] : 0.f;
  T* O = reinterpret_cast<T*>(g.out);

  // InstanceNorm-backward partials (INP): per lane the sums over its voxels of g and g (x - mean) for its 8
  // channels n0 + 8 kg + (0..7) (times rstd at the flush), g = dy if x > mean (xhat > 0; rstd > 0) else 0
  float isg[8], isgx[8], imu[8];
  int in_n = -1;
  V8<T> xin[BY];
  __shared__ float ired[INP ? 4 : 1][2][32];
  if constexpr (INP) {
#pragma unroll
    for (int k = 0; k < 8; ++k) isg[k] = isgx[k] = 0.f;
  }
  // block-wide: the sums of sample in_n -> inpart[in_n][blk][n0 + c] (fixed order: 16-lane tree, then waves 0..3)
  auto in_flush = [&]() {
   if constexpr (INP) {   // (the 1-wave LDS array of the plain instantiations is never read)
#pragma unroll
    for (int o = 1; o < 16; o <<= 1)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        isg[k] += __shfl_xor(isg[k], o, 64);
        isgx[k] += __shfl_xor(isgx[k], o, 64);
      }
    if (r16 == 0)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        ired[wave][0][8 * kg + k] = isg[k];
        ired[wave][1][8 * kg + k] = isgx[k];
      }
    __syncthreads();
    if (tid < 32) {
      const float a = ired[0][0][tid] + ired[1][0][tid] + ired[2][0][tid] + ired[3][0][tid];
      const float c = ired[0][1][tid] + ired[1][1][tid] + ired[2][1][tid] + ired[3][1][tid];
      float* p = g.inpart + (((long long)in_n * blocks_per_nt + blk) * g.Ncols + n0 + tid) * 2;
      p[0] = a;
      p[1] = c * g.inrstd[in_n * g.Ncols + n0 + tid];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) isg[k] = isgx[k] = 0.f;
   }
  };
  auto in_load = [&](const Unit& q) {   // x of the lane's 4 output voxels (consumed by the brick's epilogue)
    const T* X = reinterpret_cast<const T*>(g.inx) + (long long)q.n * vox_per_n * g.ldinx + n0 + 8 * kg;
#pragma unroll
    for (int i = 0; i < BY; ++i)
      xin[i].load(X + (long long)((q.z0 + wave) * g.H + q.y0 + i) * g.W * g.ldinx +
                  (long long)(q.x0 + r16) * g.ldinx);
  };

  // epilogue of a finished brick (ev = its accumulators, copied out of the AGPRs): lane holds channels
  // n0 + 8*kg + 4*j + (0..3) of voxel (z0 + wave, y0 + i, x0 + r16): one 16-B store per row tile
  f32x4 ev[BY][RN];
  auto epilogue = [&](const Unit& q) {
    const long long obase = (long long)q.n * vox_per_n;
    if constexpr (INP) {
      if (q.n != in_n) {   // block-uniform
        if (in_n >= 0) in_flush();
        in_n = q.n;
#pragma unroll
        for (int k = 0; k < 8; ++k) imu[k] = g.inmean[in_n * g.Ncols + n0 + 8 * kg + k];
      }
    }
#pragma unroll
    for (int i = 0; i < BY; ++i) {
      const int z = q.z0 + wave, y = q.y0 + i, x = q.x0 + r16;
      T* dst = out_at<T>(g, obase + (long long)(z * g.H + y) * g.W + x, n0 + 8 * kg);
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < RN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) o[4 * j + r] = (bf16_t)(ev[i][j][r] + bv[j][r]);
      *reinterpret_cast<bf16x8*>(dst) = o;
      if constexpr (INP) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float d = xin[i].get(k) - imu[k];
          const float gg = d > 0.f ? (float)o[k] : 0.f;
          isg[k] += gg;
          isgx[k] = fmaf(gg, d, isgx[k]);
        }
      }
    }
  };
  Unit cur = unit_of(u_begin), prev = cur;
  if constexpr (DMA) {
    set_xd(cur);
    issue_xd(0, 0, DK);
    __builtin_amdgcn_s_waitcnt(0x0f70);    // vmcnt(0): this wave's halo pieces have landed
  } else {
    set_x(cur);
    load_x(0, XK);
    store_x(0, 0, XK);
  }
  __syncthreads();
  stamp();
  int b = 0;
  for (int u = u_begin; u < u_end; ++u) {
    f32x4 acc[BY][RN];
#pragma unroll
    for (int i = 0; i < BY; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const bool unext = u + 1 < u_end;
    Unit nxt = cur;
    if (unext) {
      // next brick of the contiguous range (x fastest), stepped with uniform adds instead of divisions
      nxt.x0 += BX;
      if (nxt.x0 == g.W) {
        nxt.x0 = 0;
        nxt.y0 += BY;
        if (nxt.y0 == g.H) {
          nxt.y0 = 0;
          nxt.z0 += BZ;
          if (nxt.z0 == g.D) {
            nxt.z0 = 0;
            ++nxt.n;
          }
        }
      }
      if constexpr (DMA) set_xd(nxt);
      else set_x(nxt);
    }
    const T* Xb = Xl + b * XQ * EPQ;
    // group q = (kz, kx) = divmod(q, 3): the 6 halo rows of plane wave + kz at shift kx
    V8<T> af[2][HY];
    auto load_group = [&](V8<T> (&f)[HY], int q) {
      const int kz = q / 3, kx = q - kz * 3;
#pragma unroll
      for (int h = 0; h < HY; ++h) f[h].load(Xb + (ao[kx] + kz * RZ + h * RY) * EPQ);
    };
    stamp();
    load_group(af[0], 0);
#pragma unroll
    for (int q = 0; q < 9; ++q) {
      if (q + 1 < 9) load_group(af[(q + 1) & 1], q + 1);
      // the next brick's halo: 4 rows loaded in each of groups 0..2, 2 rows stored in each of groups 3..8,
      // so the loads' issue and the LDS writes overlap MFMAs
      if (unext) {
        if constexpr (DMA) {
          if (q < 3) issue_xd(b ^ 1, 4 * q, 4 * q + 4 < DK ? 4 * q + 4 : DK);
        } else {
          if (q < 3) load_x(4 * q, 4 * q + 4);
          else store_x(b ^ 1, 2 * (q - 3), 2 * (q - 3) + 2);
        }
      }
      if (q == 5) stamp();
      if constexpr (INP) {
        if (q == 4) in_load(cur);
      }
      __builtin_amdgcn_sched_barrier(0);   // keep the next group's reads ahead of this group's MFMAs
      // the previous brick's outputs: their VALU work and stores fill the first group's MFMA shadow
      if (q == 0 && u > u_begin) epilogue(prev);
      const int kz = q / 3, kx = q - kz * 3;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int i = 0; i < BY; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j) mfma_aw(acc[i][j], wf[kz * 9 + ky * 3 + kx][j].v, af[q & 1][i + ky].v);
    }
#pragma unroll
    for (int i = 0; i < BY; ++i) brick4_fence(acc[i][0], acc[i][1]);
    stamp();
#pragma unroll
    for (int i = 0; i < BY; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) ev[i][j] = acc[i][j];
    prev = cur;
    stamp();
    if constexpr (DMA) __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0): the next halo has landed
    __syncthreads();   // buffer b^1 is complete; buffer b is free for the brick after next
    b ^= 1;
    cur = nxt;
  }
  epilogue(prev);
  if constexpr (INP) in_flush();
}

// ------------------------------------------------- brick conv v6 (brick5 with its other work between the MFMAs)
// Stamps and the .s of brick5 (r03s, 96^3 B=2 32->32 forward, one wave per SIMD): ~8,000 cycles per brick against
// 3,456 of MFMA issue.  hipcc emitted each group's halo staging (the deferred norm's VALU work and its ds_writes),
// the next group's fragment reads and the previous brick's epilogue as blocks BETWEEN the groups' MFMA runs, and
// an MFMA run at one wave per SIMD leaves only 8 of every 16 cycles to other instructions -- when those come as a
// block, the matrix pipe idles for the whole block.  v6 is brick5's register-staged path (same layout, same
// arithmetic, bitwise the same outputs) with every group cut into 8 chunks of 3 MFMAs separated by
// sched_barrier(0), each chunk carrying a fixed share of the rest: one of the next group's 6 fragment reads, a row
// of the next brick's halo loads (groups 0-1), one 2-channel pair of a staged row's deferred norm (groups SG0..8,
// row written to LDS with its fourth pair) or one row of the previous brick's epilogue (group 0).  The steady state
// has no branches: NORM is a template parameter, out-of-volume rows are zeroed by a mask instead of a branch, the
// 40 threads without a halo column write a dummy LDS slot, the last brick re-stages itself, and the first brick's
// group-0 epilogue writes bias-only values that the next brick's epilogue (same lanes, same addresses) overwrites.
// DBG (timing probes only, wrong results): 1 = MFMAs + fragment reads only after the prologue, 2 = MFMAs only.
// INP (data gradient, no bias): the epilogue also sums the InstanceNorm-backward partials of its output, as brick5's
// INP variant (same per-lane order: bitwise the same partials); the x of a brick's output voxels is loaded in its
// group 4, its partial sums are formed in the next brick's group 1.
// F8 (forward only; mixed bf16/fp8 of config c5): the halo is staged as OCP e4m3 (the first 8 bytes of each 16-B
// quad, read by ds_read_b64), the weights come as e4m3 w * s[co] (mmseg_pack_conv3_fp8) and the MFMA is
// v_mfma_f32_16x16x32_fp8_fp8 with fp32 accumulation; the epilogue multiplies by g.wdq[co] = 1 / s[co].
template <bool NORM, int SG0 = 3, int DBG = 0, bool INP = false, bool F8 = false>
__global__ __launch_bounds__(256, 1) void conv3_brick6_kernel(GemmArgs g, int upb, int blocks_per_nt) {
  PROBE_BLOCK(false);
  using T = bf16_t;
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  constexpr int BZ = 4, BY = 4, BX = 16;
  constexpr int HZ = BZ + 2, HY = BY + 2, HX = BX + 2;
  constexpr int RY = HX * 4, RZ = HY * RY;             // quads per halo row / plane
  constexpr int XQ = HZ * RZ;                          // 2592 quads = 41.5 KB
  constexpr int RN = 2;
  constexpr int XROWS = HZ * HY;                       // 36 (z, y) halo rows
  constexpr int XK = XROWS / 3;                        // rows per thread (3 rows per pass of 216 threads)
  constexpr int NSG = 9 - SG0;                         // groups that write staged rows
  constexpr int RPG = (XK + NSG - 1) / NSG;            // rows per such group
  constexpr int PPC = RPG / 2;                         // norm pairs per chunk (4 pairs per row, 8 chunks)
  static_assert(RPG % 2 == 0 && NSG * RPG >= XK && SG0 >= 2, "SG0: 3, 6 or 7");
  constexpr int EPQ = 8;
  __shared__ __attribute__((aligned(16))) float4 lds4[2 * XQ + 64];
  T* Xl = reinterpret_cast<T*>(lds4);

  const T* Bw = reinterpret_cast<const T*>(g.b);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bz_n = g.D / BZ, by_n = g.H / BY, bx_n = g.W / BX;
  const int nbrick = (g.M / (g.D * g.H * g.W)) * bz_n * by_n * bx_n;
  const int blk_all = g.swz ? xcd_swizzle(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int nt = blk_all / blocks_per_nt, blk = blk_all - nt * blocks_per_nt;
  const int n0 = nt * 32;
  const int u_begin = blk * upb;
  const int u_end = u_begin + upb < nbrick ? u_begin + upb : nbrick;
  // INP: zero partials for the samples outside the block's unit range [n_lo, n_hi] (the consumer sums every
  // block's slot of every sample; this replaces a memset of the whole partial buffer before the launch)
  auto inp_zero = [&](int n_lo, int n_hi) {
    if constexpr (INP) {
      const int nsamp = g.M / (g.D * g.H * g.W);
      if (tid < 32 && n0 + tid < g.Ncols)
        for (int n = 0; n < nsamp; ++n)
          if (n < n_lo || n > n_hi) {
            float* p = g.inpart + (((long long)n * blocks_per_nt + blk) * g.Ncols + n0 + tid) * 2;
            p[0] = 0.f;
            p[1] = 0.f;
          }
    }
  };
  if (u_begin >= u_end || n0 >= g.Ncols) {
    inp_zero(0, -1);
    return;
  }
  const int HW = g.H * g.W;
  const int cin = 8 << g.cpg_shift;
  const int ldb = g.lda * (int)sizeof(T);
  const int vox_per_n = g.D * HW;
  const int r16 = lane & 15, kg = lane >> 4;

  V8<T> wf[F8 ? 1 : 27][RN];
  long wf8[F8 ? 27 : 1][RN];
  if constexpr (F8) {
    const long* B8 = reinterpret_cast<const long*>(g.b);
#pragma unroll
    for (int t = 0; t < 27; ++t)
#pragma unroll
      for (int j = 0; j < RN; ++j)
        wf8[t][j] = B8[(long long)(t * (cin / 8) + kg) * g.Cpad + n0 + 8 * (r16 >> 2) + 4 * j + (r16 & 3)];
#pragma unroll
    for (int t = 0; t < 27; ++t) asm volatile("s_nop 2" : "+a"(wf8[t][0]), "+a"(wf8[t][1]));
  } else {
#pragma unroll
    for (int t = 0; t < 27; ++t)
#pragma unroll
      for (int j = 0; j < RN; ++j)
        wf[t][j].load(Bw + ((long long)(t * (cin / 8) + kg) * g.Cpad + n0 + 8 * (r16 >> 2) + 4 * j + (r16 & 3)) * 8);
#pragma unroll
    for (int t = 0; t < 27; ++t) brick4_wfence(wf[t][0].v, wf[t][1].v);
  }

  const __amdgpu_buffer_rsrc_t arsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(g.a), 0, (int)((long long)(g.M / vox_per_n) * vox_per_n * ldb), 0x00020000);
  const bool xact = tid < 216;
  const int xq = tid % 72, r0 = tid / 72;
  const int hx = xq >> 2, cg = xq & 3;
  const int xlds0 = (hx * 4 + (cg ^ (((hx >> 2) & 1) << 1))) * EPQ;
  // LDS destination of staged row k in buffer b: xs0 + b * xsb + k * xsk (idle threads: a dummy slot)
  const int xs0 = xact ? xlds0 + r0 * RY * EPQ : (2 * XQ + (tid & 63)) * EPQ;
  const int xsk = xact ? 3 * RY * EPQ : 0;
  const int xsb = xact ? XQ * EPQ : 0;
  struct Unit { int n, z0, y0, x0; };
  auto unit_of = [&](int b) {
    Unit r;
    const int bx = b % bx_n; b /= bx_n;
    const int by = b % by_n; b /= by_n;
    r.z0 = (b % bz_n) * BZ;
    r.n = b / bz_n;
    r.y0 = by * BY;
    r.x0 = bx * BX;
    return r;
  };
  V8<T> xr[XK];
  uint32_t rel[XK];
#pragma unroll
  for (int k = 0; k < XK; ++k) {
    const int row = r0 + 3 * k, hz = row / HY, hy = row - hz * HY;
    rel[k] = (uint32_t)((hz * HW + hy * g.W + hx) * ldb + cg * 16);
  }
  uint32_t xo[XK], om[XK];
  float nmu[8], nrs[8];
  int norm_n = -1;
  auto set_x = [&](const Unit& q) {
    if constexpr (NORM) {
      if (q.n != norm_n) {
        norm_n = q.n;
        const int cb = q.n * cin + cg * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          nmu[j] = g.nmean[cb + j];
          nrs[j] = g.nrstd[cb + j];
        }
      }
    }
    const int xx = q.x0 - 1 + hx;
    const bool xok = xact && (unsigned)xx < (unsigned)g.W;
    const int ob = ((q.n * g.D + q.z0 - 1) * g.H + q.y0 - 1) * g.W + q.x0 - 1;
    const uint32_t base = (uint32_t)(ob * ldb);
    if (q.z0 >= 1 && q.z0 + BZ < g.D && q.y0 >= 1 && q.y0 + BY < g.H) {
#pragma unroll
      for (int k = 0; k < XK; ++k) xo[k] = xok ? base + rel[k] : 0x80000000u;
    } else {
#pragma unroll
      for (int k = 0; k < XK; ++k) {
        const int row = r0 + 3 * k, hz = row / HY, hy = row - hz * HY;
        const int zz = q.z0 - 1 + hz, yy = q.y0 - 1 + hy;
        const bool ok = xok && (unsigned)zz < (unsigned)g.D && (unsigned)yy < (unsigned)g.H;
        xo[k] = ok ? base + rel[k] : 0x80000000u;
      }
    }
#pragma unroll
    for (int k = 0; k < XK; ++k) om[k] = xo[k] != 0x80000000u ? ~0u : 0u;
  };
  auto load_row = [&](int k) { buf_load_v8<T>(xr[k], arsrc, xo[k]); };
  // deferred norm of channels 2p, 2p+1 of staged row k: in_relu_apply's operations; out-of-volume rows stay 0
  u32x4 sv[RPG];
  auto norm_pair = [&](int k, int p, u32x4& o) {
    float ha = (xr[k].get(2 * p) - nmu[2 * p]) * nrs[2 * p];
    float hb = (xr[k].get(2 * p + 1) - nmu[2 * p + 1]) * nrs[2 * p + 1];
    ha = ha > 0.f ? ha : 0.f;
    hb = hb > 0.f ? hb : 0.f;
    if constexpr (F8) {   // pairs 0, 1 -> dword 0 (low, high word), 2, 3 -> dword 1
      if (p & 1) o[p >> 1] = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(ha, hb, (int)o[p >> 1], true) & om[k];
      else o[p >> 1] = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(ha, hb, 0, false);
    } else {
      const bf16x2 h2 = {(__bf16)ha, (__bf16)hb};
      o[p] = __builtin_bit_cast(uint32_t, h2) & om[k];
    }
  };
  auto to_f8 = [&](int k, u32x4& o) {   // raw staged row (no norm) -> e4m3 (out-of-volume lanes read 0 -> 0)
#pragma unroll
    for (int d = 0; d < 2; ++d) {
      const int lo = __builtin_amdgcn_cvt_pk_fp8_f32(xr[k].get(4 * d), xr[k].get(4 * d + 1), 0, false);
      o[d] = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(xr[k].get(4 * d + 2), xr[k].get(4 * d + 3), lo, true);
    }
  };
  auto store_row = [&](int buf, int k, const u32x4& o) {
    if constexpr (F8) {
      typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
      *reinterpret_cast<u32x2*>(Xl + buf * xsb + xs0 + k * xsk) = (u32x2){o[0], o[1]};
    } else {
      *reinterpret_cast<u32x4*>(Xl + buf * xsb + xs0 + k * xsk) = o;
    }
  };
  auto stage_row = [&](int buf, int k) {   // whole row (prologue)
    u32x4 o;
    if constexpr (NORM) {
#pragma unroll
      for (int p = 0; p < 4; ++p) norm_pair(k, p, o);
    } else if constexpr (F8) {
      to_f8(k, o);
    } else {
      o = __builtin_bit_cast(u32x4, xr[k].v);
    }
    store_row(buf, k, o);
  };
  int ao[3];
#pragma unroll
  for (int kx = 0; kx < 3; ++kx) {
    const int h = r16 + kx;
    ao[kx] = wave * RZ + h * 4 + (kg ^ (((h >> 2) & 1) << 1));
  }
  float bv[RN][4], dq[F8 ? RN : 1][4];
#pragma unroll
  for (int j = 0; j < RN; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      bv[j][r] = g.bias ? g.bias[n0 + 8 * kg + 4 * j + r] : 0.f;
      if constexpr (F8) dq[j][r] = g.wdq[n0 + 8 * kg + 4 * j + r];
    }

  f32x4 ev[BY][RN];
#pragma unroll
  for (int i = 0; i < BY; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) ev[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // row i of a finished brick: lane holds channels n0 + 8 kg + 4 j + (0..3) of voxel (z0 + wave, y0 + i, x0 + r16)
  bf16x8 eo[BY];   // the stored rows (INP: their partial sums follow one group later)
  auto epi_row = [&](const Unit& q, int i) {
    const long long obase = (long long)q.n * vox_per_n;
    const int z = q.z0 + wave, y = q.y0 + i, x = q.x0 + r16;
    T* dst = out_at<T>(g, obase + (long long)(z * g.H + y) * g.W + x, n0 + 8 * kg);
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if constexpr (F8) eo[i][4 * j + r] = (bf16_t)fmaf(ev[i][j][r], dq[j][r], bv[j][r]);
        else eo[i][4 * j + r] = (bf16_t)(ev[i][j][r] + bv[j][r]);
      }
    *reinterpret_cast<bf16x8*>(dst) = eo[i];
  };
  // InstanceNorm-backward partials (INP): per lane the sums over its voxels of g and g (x - mean) for channels
  // n0 + 8 kg + (0..7), g = dy if x > mean else 0 (times rstd at the flush); the first brick's epilogue runs on
  // zeroed accumulators and x and adds 0
  __shared__ float ired[INP ? 4 : 1][2][32];
  float isg[8], isgx[8], imu[8];
  int in_n = -1;
  V8<T> xin[BY];
  if constexpr (INP) {
#pragma unroll
    for (int k = 0; k < 8; ++k) isg[k] = isgx[k] = imu[k] = 0.f;
#pragma unroll
    for (int i = 0; i < BY; ++i) xin[i].zero();
  }
  auto in_flush = [&]() {
   if constexpr (INP) {   // (the 1-wave LDS array of the plain instantiations is never read)   // block-wide, fixed order: 16-lane tree, then waves 0..3
#pragma unroll
    for (int o = 1; o < 16; o <<= 1)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        isg[k] += __shfl_xor(isg[k], o, 64);
        isgx[k] += __shfl_xor(isgx[k], o, 64);
      }
    if (r16 == 0)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        ired[wave][0][8 * kg + k] = isg[k];
        ired[wave][1][8 * kg + k] = isgx[k];
      }
    __syncthreads();
    if (tid < 32) {
      const float a = ired[0][0][tid] + ired[1][0][tid] + ired[2][0][tid] + ired[3][0][tid];
      const float c = ired[0][1][tid] + ired[1][1][tid] + ired[2][1][tid] + ired[3][1][tid];
      float* p = g.inpart + (((long long)in_n * blocks_per_nt + blk) * g.Ncols + n0 + tid) * 2;
      p[0] = a;
      p[1] = c * g.inrstd[in_n * g.Ncols + n0 + tid];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) isg[k] = isgx[k] = 0.f;
   }
  };
  auto in_begin = [&](const Unit& q) {   // block-uniform: the sample of the epilogue's brick
    if constexpr (INP) {
      if (q.n != in_n) {
        if (in_n >= 0) in_flush();
        in_n = q.n;
#pragma unroll
        for (int k = 0; k < 8; ++k) imu[k] = g.inmean[in_n * g.Ncols + n0 + 8 * kg + k];
      }
    }
  };
  auto in_load_row = [&](const Unit& q, int i) {   // x of the lane's output voxel of row i
    const T* X = reinterpret_cast<const T*>(g.inx) + (long long)q.n * vox_per_n * g.ldinx + n0 + 8 * kg;
    xin[i].load(X + (long long)((q.z0 + wave) * g.H + q.y0 + i) * g.W * g.ldinx + (long long)(q.x0 + r16) * g.ldinx);
  };
  auto epi_inp = [&](int i, int half) {
#pragma unroll
    for (int k = 4 * half; k < 4 * half + 4; ++k) {
      const float d = xin[i].get(k) - imu[k];
      const float gg = d > 0.f ? (float)eo[i][k] : 0.f;
      isg[k] += gg;
      isgx[k] = fmaf(gg, d, isgx[k]);
    }
  };

  Unit cur = unit_of(u_begin), prev = cur;
  set_x(cur);
#pragma unroll
  for (int k = 0; k < XK; ++k) load_row(k);
#pragma unroll
  for (int k = 0; k < XK; ++k) stage_row(0, k);
  __syncthreads();
  int b = 0;
  for (int u = u_begin; u < u_end; ++u) {
    f32x4 acc[BY][RN];   // (first written by the C = 0 MFMAs of group 0)
    Unit nxt = cur;
    if (u + 1 < u_end) {   // (the last brick re-stages itself into the idle buffer)
      nxt.x0 += BX;
      if (nxt.x0 == g.W) {
        nxt.x0 = 0;
        nxt.y0 += BY;
        if (nxt.y0 == g.H) {
          nxt.y0 = 0;
          nxt.z0 += BZ;
          if (nxt.z0 == g.D) {
            nxt.z0 = 0;
            ++nxt.n;
          }
        }
      }
    }
    set_x(nxt);
    in_begin(prev);
    const T* Xb = Xl + b * XQ * EPQ;
    V8<T> af[F8 ? 1 : 2][HY];
    long af8[F8 ? 2 : 1][HY];
#pragma unroll
    for (int h = 0; h < HY; ++h) {
      if constexpr (F8) af8[0][h] = *reinterpret_cast<const long*>(Xb + (ao[0] + h * RY) * EPQ);
      else af[0][h].load(Xb + (ao[0] + h * RY) * EPQ);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 9; ++q) {
      const int kz = q / 3, kx = q - kz * 3;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        if (q + 1 < 9 && c < HY && DBG < 2) {     // fragment c of the next group
          const int qn = q + 1, kzn = qn / 3, kxn = qn - kzn * 3;
          if constexpr (F8) af8[qn & 1][c] = *reinterpret_cast<const long*>(Xb + (ao[kxn] + kzn * RZ + c * RY) * EPQ);
          else af[qn & 1][c].load(Xb + (ao[kxn] + kzn * RZ + c * RY) * EPQ);
        }
        if (q == 0 && DBG == 0) {
          load_row(c);                  // next brick's halo rows 0..7
          if ((c & 1) == 0) epi_row(prev, c >> 1);
        }
        if (q == 1 && c < XK - 8 && DBG == 0) load_row(8 + c);
        if constexpr (INP) {
          if (q == 1 && DBG == 0) epi_inp(c >> 1, c & 1);
          if (q == 4 && c < BY && DBG == 0) in_load_row(cur, c);
        }
        if (q >= SG0 && DBG == 0) {
#pragma unroll
          for (int pp = 0; pp < PPC; ++pp) {
            const int pi = c * PPC + pp;            // pair index inside the group: row slot pi / 4, pair pi % 4
            const int k = (q - SG0) * RPG + pi / 4;
            if (k < XK) {
              if constexpr (NORM) norm_pair(k, pi % 4, sv[pi / 4]);
              else if constexpr (F8) { if (pi % 4 == 0) to_f8(k, sv[pi / 4]); }
              else if (pi % 4 == 0) sv[pi / 4] = __builtin_bit_cast(u32x4, xr[k].v);
              if (pi % 4 == 3) store_row(b ^ 1, k, sv[pi / 4]);
            }
          }
        }
#pragma unroll
        for (int m = 3 * c; m < 3 * c + 3; ++m) {
          const int ky = m >> 3, i = (m >> 1) & 3, j = m & 1;
          if constexpr (F8) {
            if (q == 0 && ky == 0) mfma_aw80(acc[i][j], wf8[kx][j], af8[0][i]);
            else mfma_aw8(acc[i][j], wf8[kz * 9 + ky * 3 + kx][j], af8[q & 1][i + ky]);
          } else {
            if (q == 0 && ky == 0) mfma_aw0(acc[i][j], wf[kx][j].v, af[0][i].v);
            else mfma_aw(acc[i][j], wf[kz * 9 + ky * 3 + kx][j].v, af[q & 1][i + ky].v);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // one MFMA-result hazard fence over all 8 accumulators before they are copied
    asm volatile("s_nop 7\n\ts_nop 7" : "+a"(acc[0][0]), "+a"(acc[0][1]), "+a"(acc[1][0]), "+a"(acc[1][1]),
                 "+a"(acc[2][0]), "+a"(acc[2][1]), "+a"(acc[3][0]), "+a"(acc[3][1]));
#pragma unroll
    for (int i = 0; i < BY; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) ev[i][j] = acc[i][j];
    prev = cur;
    __syncthreads();   // buffer b^1 is complete; buffer b is free for the brick after next
    b ^= 1;
    cur = nxt;
  }
  in_begin(prev);
#pragma unroll
  for (int i = 0; i < BY; ++i) {
    epi_row(prev, i);
    if constexpr (INP) {
      epi_inp(i, 0);
      epi_inp(i, 1);
    }
  }
  if constexpr (INP) {
    in_flush();
    inp_zero(u_begin / (nbrick / (g.M / vox_per_n)), in_n);
  }
  PROBE_BLOCK(true);
}

// ------------------------------------- runtime-brick conv (small volumes)
// conv3_brick2_kernel for volumes whose sides are not multiples of 8 (the
// 12^3 and 6^3 levels): the brick (bz, by, bx), <= 256 voxels, is chosen on the
// host among divisors of (D, H, W), and the 27*Cin reduction can be split over
// 32-channel chunks (fp32 partials [ks][M][Ncols] + gemm_splitk_reduce) so that
// a handful of bricks still fills the chip.  Row r of the block (wave*64 + i*16
// + lane%16) is brick voxel r; rows >= bz*by*bx compute garbage and are never
// stored.
constexpr int BR_MAXHV = 640;   // halo voxels staged per block (host guarantees)
// halo image quads available (host guarantees (bz+2)(by+2)((bx+2)*QV+2) <= this): 40 KB bf16 / 80 KB f32
__host__ __device__ constexpr int br_xq(int tsize) { return tsize == 2 ? 2560 : 5120; }

// CB* > 0: the brick is known at compile time (6x6x6 at the 12^3 / 6^3 levels), so the halo / epilogue index
// arithmetic divides by constants (mul-shift) instead of runtime integer divisions, which at one 32-channel
// chunk per block were most of the kernel's VALU work (8.6 VALU instructions per MFMA, rocprofv3 r02).
// B32 (bf16): the halo staged with 32-bit offset buffer loads, out-of-volume lanes reading zeros (conv3_brick2's B32).
// KW = 2 (12^3 / 6^3, r05): 512-thread blocks whose two 256-thread halves split the block's 32-channel chunks
// (half 0 the first ceil(n/2), half 1 the rest), each with its own halo / weight stage buffers, in lockstep through
// the same barriers; half 1's accumulators are added to half 0's through LDS (fixed order) before the epilogue.
// At these levels a launch has ~256 blocks, one per CU, so the KW = 1 form runs ONE wave per SIMD and nothing
// hides a wave's staging and LDS latency; two K-halves give every SIMD a second wave without a global split.
template <typename T, int BN, int CBZ = 0, int CBY = 0, int CBX = 0, int DBG = 0, bool PF = false, bool B32 = false,
          int KW = 1>
__global__ __launch_bounds__(256 * KW, (sizeof(T) == 2 && KW == 1) ? 2 : 1) void conv3_brickr_kernel(
    GemmArgs g, int bz_rt, int by_rt, int bx_rt, long long* dbg = nullptr) {
  const int bz = CBZ > 0 ? CBZ : bz_rt, by = CBY > 0 ? CBY : by_rt, bx = CBX > 0 ? CBX : bx_rt;
  // DBG 4: every block's (realtime, memtime) at start / end, block 0 wave 0's per-phase memtime stamps
  int dn = 0;
  auto stamp = [&]() {
    if constexpr (DBG == 4) {
      if (blockIdx.x == 0 && threadIdx.x == 0 && dn < 64) dbg[4 * 4096 + dn++] = (long long)__builtin_amdgcn_s_memtime();
    }
  };
  if constexpr (DBG == 4) {
    if (threadIdx.x == 0) {
      dbg[4 * blockIdx.x + 0] = (long long)__builtin_amdgcn_s_memrealtime();
      dbg[4 * blockIdx.x + 1] = (long long)__builtin_amdgcn_s_memtime();
    }
  }
  stamp();
  using L = Brick2Layout<T>;
  constexpr int RM = 4, RN = BN / 16;
  constexpr int XQ = br_xq(sizeof(T));
  constexpr int WQ = 9 * BN * L::QV;
  constexpr int EQ = (256 * (BN + 4) * 4 + 15) / 16;   // fp32 epilogue tile
  constexpr int RQ = KW > 1 ? 256 * BN / 4 : 0;           // half 1's accumulators (fp32), after the epilogue tile
  constexpr int LQ = (KW * (XQ + WQ)) > (EQ + RQ) ? (KW * (XQ + WQ)) : (EQ + RQ);
  __shared__ __attribute__((aligned(16))) float4 lds4[LQ];
  const int half = KW > 1 ? (int)(threadIdx.x >> 8) : 0;
  T* Xl = reinterpret_cast<T*>(lds4 + half * (XQ + WQ));
  T* Wl = reinterpret_cast<T*>(lds4 + half * (XQ + WQ) + XQ);
  constexpr int EPQ = 16 / sizeof(T);
  constexpr int X_PER = (BR_MAXHV * 4 + 255) / 256;
  constexpr int W_ITEMS = 9 * BN * 4;
  constexpr int W_PER = (W_ITEMS + 255) / 256;

  const int HX = bx + 2, HY = by + 2, HZ = bz + 2;
  const int RY = HX * L::QV + 2, RZ = HY * RY;
  const int HV = HZ * HY * HX;
  const int X_ITEMS = HV * 4;
  const int rows = bz * by * bx;

  const T* A = reinterpret_cast<const T*>(g.a);
  const T* Bw = reinterpret_cast<const T*>(g.b);
  const int tid = threadIdx.x & 255, lane = tid & 63, wave = tid >> 6;
  const int bz_n = g.D / bz, by_n = g.H / by, bx_n = g.W / bx;
  const int nbrick = (g.M / (g.D * g.H * g.W)) * bz_n * by_n * bx_n;
  const int nt_n = (g.Ncols + BN - 1) / BN;
  const int tile = g.swz ? xcd_swizzle(blockIdx.x, nbrick * nt_n * g.ksplit) : (int)blockIdx.x;
  int bidx = tile % nbrick;
  const int nt = (tile / nbrick) % nt_n;
  const int ks = tile / (nbrick * nt_n);
  const int bxi = bidx % bx_n; bidx /= bx_n;
  const int byi = bidx % by_n; bidx /= by_n;
  const int bzi = bidx % bz_n;
  const int n = bidx / bz_n;
  const int z0 = bzi * bz, y0 = byi * by, x0 = bxi * bx;
  const long long HW = (long long)g.H * g.W;
  const long long nbase = (long long)n * g.D * HW;
  const int grp = g.grp_n > 0 ? n / g.grp_n : 0;     // grouped launch: this brick's weight / bias group
  if (grp) Bw += (long long)grp * g.w_gstride;
  const float* biasp = (g.bias && grp) ? g.bias + grp * g.b_gstride : g.bias;
  const int n0 = nt * BN;
  const int cin = 8 << g.cpg_shift;
  const int nchunk = gemm_nchunk(g);
  const int cps = (nchunk + g.ksplit - 1) / g.ksplit;
  const int cb0 = ks * cps;
  const int ce0 = cb0 + cps < nchunk ? cb0 + cps : nchunk;
  // KW = 2: this half's chunks of the block's range (half 0 takes the larger share when it is odd)
  const int cmid = cb0 + (ce0 - cb0 + 1) / 2;
  const int c_begin = KW > 1 && half ? cmid : cb0;
  const int c_end = KW > 1 ? (half ? ce0 : cmid) : ce0;
  // iterations every thread of the block runs (the barriers inside the loop are block-wide): half 0's count
  const int n_iter = ((KW > 1 ? cmid : ce0) - cb0) * 3;

  V8<T> xr[X_PER], wr[W_PER];
  const int nvox = n * g.D * g.H * g.W;   // (B32 only: the host checked the extent)
  const __amdgpu_buffer_rsrc_t arsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(g.a), 0, B32 ? (int)((long long)g.M * g.lda * (int)sizeof(T)) : 0, 0x00020000);
  auto load_x = [&](int c) {
#pragma unroll
    for (int k = 0; k < X_PER; ++k) {
      const int e = tid + k * 256;
      if (e < X_ITEMS) {
        const int h = e >> 2, cg = e & 3;
        const int hx = h % HX, t = h / HX;
        const int hy = t % HY, hz = t / HY;
        const int z = z0 - 1 + hz, y = y0 - 1 + hy, x = x0 - 1 + hx;
        const bool ok = (unsigned)z < (unsigned)g.D && (unsigned)y < (unsigned)g.H && (unsigned)x < (unsigned)g.W;
        if constexpr (B32) {
          const uint32_t off = ok ? (uint32_t)(((nvox + (z * g.H + y) * g.W + x) * g.lda + c * CK + cg * 8) *
                                               (int)sizeof(T))
                                  : 0x80000000u;
          buf_load_v8<T>(xr[k], arsrc, off);   // out-of-volume lanes read zeros
        } else {
          if (ok)
            xr[k].load(A + (nbase + z * HW + (long long)y * g.W + x) * g.lda + c * CK + cg * 8);
          else
            xr[k].zero();
        }
      }
    }
  };
  auto store_x = [&]() {
#pragma unroll
    for (int k = 0; k < X_PER; ++k) {
      const int e = tid + k * 256;
      if (e < X_ITEMS) {
        const int h = e >> 2, cg = e & 3;
        const int hx = h % HX, t = h / HX;
        const int hy = t % HY, hz = t / HY;
        xr[k].store(Xl + (hz * RZ + hy * RY + hx * L::QV + cg * L::QG) * EPQ);
      }
    }
  };
  auto load_w = [&](int c, int kz) {
#pragma unroll
    for (int k = 0; k < W_PER; ++k) {
      const int e = tid + k * 256;
      if (e < W_ITEMS) {
        const int cg = e & 3, q = e >> 2;
        const int col = q % BN, t9 = q / BN;
        const int kgi = (kz * 9 + t9) * (cin / 8) + c * 4 + cg;
        wr[k].load(Bw + ((long long)kgi * g.Cpad + n0 + col) * 8);
      }
    }
  };
  auto store_w = [&]() {
#pragma unroll
    for (int k = 0; k < W_PER; ++k) {
      const int e = tid + k * 256;
      if (e < W_ITEMS) {
        const int cg = e & 3, q = e >> 2;
        wr[k].store(Wl + (q * L::QV + (cg ^ w2_swz(q)) * L::QG) * EPQ);
      }
    }
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int r16 = lane & 15, kg = lane >> 4;
  int aq[RM];
#pragma unroll
  for (int i = 0; i < RM; ++i) {
    int rr = wave * 64 + i * 16 + r16;
    if (rr >= rows) rr = 0;   // padding rows read voxel 0's halo (never stored)
    const int rx = rr % bx, t = rr / bx;
    const int ry = t % by, rz = t / by;
    aq[i] = rz * RZ + ry * RY + rx * L::QV + kg * L::QG;
  }
  int bq[RN];
#pragma unroll
  for (int j = 0; j < RN; ++j) {
    const int col = j * 16 + r16;
    bq[j] = col * L::QV + (kg ^ w2_swz(col)) * L::QG;
  }

  const int st_begin = c_begin * 3, st_end = c_end * 3;
  if (st_begin < st_end) {
    load_x(c_begin);
    load_w(c_begin, 0);
    store_x();
    store_w();
  }
  __syncthreads();
  stamp();
  for (int it = 0; it < n_iter; ++it) {
    const int st = st_begin + it;
    const bool active = st < st_end;   // (KW = 2: half 1 may own one chunk fewer; it still joins every barrier)
    const int kz = st % 3;
    const int sn = st + 1;
    const bool more = sn < st_end;
    const int cn = sn / 3, kzn = sn - cn * 3;
    if (more && DBG != 1) {
      load_w(cn, kzn);
      if (kzn == 0) load_x(cn);
    }
    if (!active) {
    } else if constexpr (PF) {
      // fragments of tap t+1 are read while tap t's MFMAs run: at one block per CU (one wave per SIMD) nothing
      // else hides the LDS latency (s_memtime: ~4,200 cycles per 9-tap stage against 2,304 of MFMA)
      V8<T> af[2][RM], bf[2][RN];
      auto rd = [&](int t9, int b) {
        const int ky = t9 / 3, kx = t9 - ky * 3;
        const int hoff = kz * RZ + ky * RY + kx * L::QV;
#pragma unroll
        for (int j = 0; j < RN; ++j) bf[b][j].load(Wl + (t9 * BN * L::QV + bq[j]) * EPQ);
#pragma unroll
        for (int i = 0; i < RM; ++i) af[b][i].load(Xl + (aq[i] + hoff) * EPQ);
      };
      rd(0, 0);
#pragma unroll
      for (int t9 = 0; t9 < 9; ++t9) {
        if (t9 < 8) rd(t9 + 1, (t9 + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j) mfma_step<T>(acc[i][j], af[t9 & 1][i], bf[t9 & 1][j]);
      }
    } else
#pragma unroll
    for (int t9 = 0; t9 < 9; ++t9) {
      const int ky = t9 / 3, kx = t9 - ky * 3;
      const int hoff = kz * RZ + ky * RY + kx * L::QV;
      V8<T> af[RM], bf[RN];
#pragma unroll
      for (int j = 0; j < RN; ++j) bf[j].load(Wl + (t9 * BN * L::QV + bq[j]) * EPQ);
#pragma unroll
      for (int i = 0; i < RM; ++i) af[i].load(Xl + (aq[i] + hoff) * EPQ);
      if (DBG == 2) {
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j) acc[i][j][0] += (float)af[i].get(0) * (float)bf[j].get(1);
      } else {
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j) mfma_step<T>(acc[i][j], af[i], bf[j]);
      }
    }
    stamp();
    __syncthreads();
    stamp();
    if (more && DBG != 3) {
      store_w();
      if (kzn == 0) store_x();
    }
    if (KW > 1 || (more && DBG != 3)) __syncthreads();   // (KW = 2: the halves' `more` may differ)
    stamp();
  }

  // KW = 2: half 1's accumulators added to half 0's (the loop ended with a barrier: the stage buffers are free)
  if constexpr (KW > 1) {
    f32x4* R4 = reinterpret_cast<f32x4*>(lds4 + EQ);
    if (half) {
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j) R4[((wave * RM + i) * RN + j) * 64 + lane] = acc[i][j];
    }
    __syncthreads();
    if (!half) {
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j) {
          const f32x4 o = R4[((wave * RM + i) * RN + j) * 64 + lane];
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] += o[r];
        }
    }
  }
  // epilogue through LDS: rows < bz*by*bx only (KW = 2: half 0 fills the tile, all 512 threads store it)
  auto row_vox = [&](int rr) {
    const int rx = rr % bx, t = rr / bx;
    const int ry = t % by, rz = t / by;
    return nbase + (z0 + rz) * HW + (long long)(y0 + ry) * g.W + (x0 + rx);
  };
  const int etid = threadIdx.x;
  constexpr int ET = 256 * KW;
  if (g.ksplit == 1) {
    T* El = reinterpret_cast<T*>(lds4);
    constexpr int EP = BN + 8;
    if (!half) {
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int col = j * 16 + r16;
        const float bv = (biasp && n0 + col < g.Ncols) ? biasp[n0 + col] : 0.f;
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) El[(wave * 64 + i * 16 + kg * 4 + r) * EP + col] = from_f<T>(acc[i][j][r] + bv);
      }
    }
    __syncthreads();
    if (KW == 1 && g.stats) {
      float* red = reinterpret_cast<float*>(El + 256 * EP);
      const long long brick = (long long)n * (bz_n * by_n * bx_n) + ((long long)bzi * by_n + byi) * bx_n + bxi;
      brick_in_stats<T, BN>(El, EP, rows, red, g.stats, brick, n0, g.Ncols);
    }
    T* O = reinterpret_cast<T*>(g.out);
    constexpr int CG = BN / 8;
    for (int e = etid; e < rows * CG; e += ET) {
      const int rr = e / CG, cg = e % CG;
      const int col = n0 + cg * 8;
      if (col < g.Ncols) {
        V8<T> o;
        o.load(El + rr * EP + cg * 8);
        o.store(out_at<T>(g, row_vox(rr), col));
      }
    }
  } else {
    float* El = reinterpret_cast<float*>(lds4);
    constexpr int EP = BN + 4;
    if (!half) {
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int col = j * 16 + r16;
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) El[(wave * 64 + i * 16 + kg * 4 + r) * EP + col] = acc[i][j][r];
      }
    }
    __syncthreads();
    constexpr int CG = BN / 4;
    for (int e = etid; e < rows * CG; e += ET) {
      const int rr = e / CG, cg = e % CG;
      const int col = n0 + cg * 4;
      if (col < g.Ncols) {
        const float4 v = *reinterpret_cast<const float4*>(El + rr * EP + cg * 4);
        *reinterpret_cast<float4*>(g.part + ((long long)ks * g.M + row_vox(rr)) * g.Ncols + col) = v;
      }
    }
  }
  if constexpr (DBG == 4) {
    stamp();
    __syncthreads();
    if (threadIdx.x == 0) {
      dbg[4 * blockIdx.x + 2] = (long long)__builtin_amdgcn_s_memrealtime();
      dbg[4 * blockIdx.x + 3] = (long long)__builtin_amdgcn_s_memtime();
    }
  }
}

// Host-side choice of the CONV3 kernel (shared by the launcher and mmseg_conv3_splits).
struct Conv3Plan {
  int kind;          // 0 per-lane gather GEMM, 1 brick2, 2 runtime brick
  int bz, by, bx;    // kind 2
  int ks;            // splits the plan wants (kind 2: over 32-channel chunks)
  int bn;            // kind 2 column tile
};

// force_r: the runtime-brick kernel even where the (4, 8, 8)-brick family fits -- the modality-grouped launches,
// whose per-group weights only the runtime-brick kernel reads (24^3 with MMSEG_GROUP_FORCE_R)
Conv3Plan plan_conv3(int M, int Ncols, int cin, int D, int H, int W, int lda, int ldo, int tsize,
                     bool force_r = false) {
  Conv3Plan p{0, 0, 0, 0, 1, 32};
  bool k1_ok = false;   // the brick2 family can take the shape (used when the runtime brick cannot)
  const int brick = knob("MMSEG_BRICK", 2);
  const bool base_ok = cin % CK == 0 && lda % 8 == 0 && ldo % 8 == 0 && Ncols % 32 == 0;
  // 48-column multiples (SwinUNETR's feature_size 48) run the brick2 kernel with 48-column tiles
  const bool ok48 = cin % CK == 0 && lda % 8 == 0 && ldo % 8 == 0 && Ncols % 48 == 0;
  if (!force_r && brick == 2 && (base_ok || ok48) && D % 4 == 0 && H % B2_Y == 0 && W % B2_X == 0) {
    // a brick2-family launch has one block per (4x8x8 brick, column tile): at SwinUNETR's 8^3 / 16^3 levels
    // (384 / 192 channels) that is 12-48 blocks for the whole chip (brick3 at 75-290 TF/s, r05m).  Below
    // MMSEG_BRICK2_MINUNITS such shapes take the runtime-brick kernel, whose chunk splits fill the CUs.
    const long long units = (long long)(M / (D * H * W)) * (D / 4) * (H / B2_Y) * (W / B2_X) *
                            ((Ncols + 63) / 64);
    if (!(base_ok && units < knob("MMSEG_BRICK2_MINUNITS", 128))) {
      p.kind = 1;
      return p;
    }
    k1_ok = true;
  }
  if (brick >= 2 && base_ok) {
    int best = 0;
    for (int bz = 1; bz <= D && bz <= 8; ++bz) {
      if (D % bz) continue;
      for (int by = 1; by <= H && by <= 16; ++by) {
        if (H % by) continue;
        for (int bx = 1; bx <= W && bx <= 16; ++bx) {
          if (W % bx) continue;
          const int rows = bz * by * bx;
          const int halo = (bz + 2) * (by + 2) * (bx + 2);
          const int hq = (bz + 2) * (by + 2) * ((bx + 2) * 2 * tsize + 2);
          if (rows > 256 || halo > BR_MAXHV || hq > br_xq(tsize)) continue;
          const int score = rows * 4 + (bx % 8 == 0 ? 2 : 0) + (by % 8 == 0 ? 1 : 0);
          // ties go to the smaller halo (12^3: 6x6x6, 512 halo voxels and the compile-time kernel, over 3x6x12)
          const bool tie_better = score == best && halo < (p.bz + 2) * (p.by + 2) * (p.bx + 2);
          if (score > best || tie_better) {
            best = score;
            p.bz = bz; p.by = by; p.bx = bx;
          }
        }
      }
    }
    if (best >= 64 * 4) {   // at least a quarter of the 256-row tile in use
      p.kind = 2;
      p.bn = (tsize == 2 && Ncols % 64 == 0) ? 64 : 32;
      const int nb = (M / (D * H * W)) * (D / p.bz) * (H / p.by) * (W / p.bx);
      // 32-column tiles where 64-column ones leave fewer than 256 blocks: twice the blocks instead of a chunk split
      // (no fp32 partials, no reduce launch); 12^3 / 6^3 grouped: 2-8 us per launch (r04v convbench), -0.02 ms/step
      if (p.bn == 64 && nb * (Ncols / 64) < 256) p.bn = 32;
      const int nt = (Ncols + p.bn - 1) / p.bn;
      const int nchunk = cin / CK;
      const int slots = knob("MMSEG_BRICKR_SLOTS", 256);   // 512 measured 2-10 % slower at 12^3 / 6^3 (r02)
      int ks = (slots + nb * nt - 1) / (nb * nt);
      if (ks > nchunk) ks = nchunk;
      if (ks < 1) ks = 1;
      const int cps = (nchunk + ks - 1) / ks;
      p.ks = (nchunk + cps - 1) / cps;
      return p;
    }
  }
  if (k1_ok) p.kind = 1;
  return p;
}

// True when launch_gemm<bf16, CONV3> runs conv3_brick5_kernel for this shape (the only conv kernel that
// applies a deferred InstanceNorm + ReLU to its A source): the conditions of its branch in launch_gemm and of
// every branch taken before it.
bool brick5_selected(const GemmArgs& g, int tsize) {
  if (tsize != 2 || g.ksplit != 1 || g.stats != nullptr) return false;
  const Conv3Plan plan = plan_conv3(g.M, g.Ncols, 8 << g.cpg_shift, g.D, g.H, g.W, g.lda, g.ldo, tsize);
  if (plan.kind != 1) return false;
  const int nb1 = (g.M / (g.D * g.H * g.W)) * (g.D / 4) * (g.H / B2_Y) * (g.W / B2_X);
  const int min_blocks = knob("MMSEG_BRICK2_MINBLK", 512);
  const bool v3 = (long long)g.M * g.lda * 2LL < (1LL << 31);
  const bool wide = g.Ncols % 64 == 0 && nb1 * (g.Ncols / 64) >= min_blocks;
  if (!v3 || g.Ncols % 32 != 0 || gemm_nchunk(g) != 1 || wide) return false;
  return g.H % 4 == 0 && g.W % 16 == 0 && g.ldo % 8 == 0 && (reinterpret_cast<uintptr_t>(g.out) & 15) == 0;
}

// Every column tile of a conv launch reads weight columns [n0, n0 + BN) of the packed image [KGp][Cpad][8]: all of
// them must lie inside the image's pitch Cpad (the r05f GPU fault: a 192-column tile over a 96-column layer's
// 128-column image read 64 columns past it).  Checked on the host before each launch, with the kernel's name noted.
inline bool tile_in_pitch(const GemmArgs& g, int BN) { return (long long)((g.Ncols + BN - 1) / BN) * BN <= g.Cpad; }
#define MMSEG_TILE(G, NAME, BN)                                                                                   \
  do {                                                                                                           \
    MMSEG_REQUIRE(tile_in_pitch((G), (BN)), "%s: %d-column tiles over %d columns exceed the packed pitch %d", \
                  (const char*)(NAME), (int)(BN), (G).Ncols, (G).Cpad);                                          \
    mmseg::note_kernel(NAME);                                                                                    \
  } while (0)

// The W % 16 one-chunk 32-column conv: brick6 (forward, deferred-norm forward, e4m3 forward, and the data gradient
// with the InstanceNorm-backward partials); brick5 only for a partials launch with a bias term (never on the
// engine's path: a data gradient has no bias).  Returns the bricks per block.
int launch_brick5(const GemmArgs& g, hipStream_t s) {
  const int nt_n = g.Ncols / 32;
  const int per_nt = std::max(1, knob("MMSEG_BRICK4_BLOCKS", 256) / nt_n);
  const int nb5 = (g.M / (g.D * g.H * g.W)) * (g.D / 4) * (g.H / 4) * (g.W / 16);
  const int upb5 = ceil_div(nb5, std::min(per_nt, nb5));
  const int bpn5 = ceil_div(nb5, upb5);
  const dim3 grid(bpn5 * nt_n), block(256);
  if (g.wdq) {   // e4m3 forward (mmseg_conv3_fwd_fp8)
    MMSEG_TILE(g, "conv3_brick6_kernel<BN32,F8>", 32);
    if (g.nmean) MMSEG_LAUNCH((conv3_brick6_kernel<true, 6, 0, false, true>), grid, block, 0, s, g, upb5, bpn5);
    else MMSEG_LAUNCH((conv3_brick6_kernel<false, 6, 0, false, true>), grid, block, 0, s, g, upb5, bpn5);
    return upb5;
  }
  if (g.inpart) {   // samples a block does not touch keep zero partials
    if (!g.bias) {   // (brick6 writes those zeros itself)
      MMSEG_TILE(g, "conv3_brick6_kernel<BN32,INP>", 32);
      MMSEG_LAUNCH((conv3_brick6_kernel<false, 6, 0, true>), grid, block, 0, s, g, upb5, bpn5);
      return upb5;
    }
    MMSEG_TILE(g, "conv3_brick5_kernel<BN32>", 32);
    hipMemsetAsync(g.inpart, 0, sizeof(float) * 2 * (size_t)(g.M / (g.D * g.H * g.W)) * bpn5 * g.Ncols, s);
    MMSEG_LAUNCH((conv3_brick5_kernel<false, true, true>), grid, block, 0, s, g, upb5, bpn5, nullptr);
    return upb5;
  }
  MMSEG_TILE(g, "conv3_brick6_kernel<BN32>", 32);
  if (g.nmean)
    MMSEG_LAUNCH((conv3_brick6_kernel<true, 6>), grid, block, 0, s, g, upb5, bpn5);
  else
    MMSEG_LAUNCH((conv3_brick6_kernel<false, 6>), grid, block, 0, s, g, upb5, bpn5);
  return upb5;
}

// 4 consecutive columns per thread in gemm_splitk_reduce (for the transposed conv: 4 channels of one child voxel,
// Cout % 4 == 0)
template <int MODE>
__host__ __device__ __forceinline__ bool splitk_vec(const GemmArgs& g) {
  const bool al = (g.Ncols & 3) == 0 && (g.ldo & 3) == 0 && (reinterpret_cast<uintptr_t>(g.part) & 15) == 0;
  return MODE == MODE_CONVT_FWD ? al && ((g.Ncols >> 3) & 3) == 0 : al;
}
template <int MODE>
int splitk_reduce_blocks(const GemmArgs& g) {
  const long long total = (long long)g.M * g.Ncols;
  return ceil_div(splitk_vec<MODE>(g) ? (total + 3) / 4 : total, 256);
}

// Fixed-order split-K reduction for the forward GEMM: out = sum_k part[k] (+bias).
template <typename T, int MODE>
__global__ void gemm_splitk_reduce(GemmArgs g) {
  long long total = (long long)g.M * g.Ncols;
  if (MODE == MODE_CONVT_FWD && splitk_vec<MODE>(g)) {
    // 4 channels of one child voxel per thread: one child-index computation per 4 values (was one per value)
    const long long idx4 = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (idx4 >= total) return;
    const long long row = idx4 / g.Ncols;
    const int col = (int)(idx4 - row * g.Ncols);
    const int Cout = g.Ncols >> 3, t = col / Cout, co = col - t * Cout;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    const float4* p = reinterpret_cast<const float4*>(g.part + idx4);
    const long long st = total / 4;
#pragma unroll 4
    for (int k = 0; k < g.ksplit; ++k) {
      const float4 a = p[(long long)k * st];
      v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
    }
    if (g.bias) {
      v.x += g.bias[co]; v.y += g.bias[co + 1]; v.z += g.bias[co + 2]; v.w += g.bias[co + 3];
    }
    T* O = reinterpret_cast<T*>(g.out) + convt_child(row, t, g) * g.ldo + co;
    O[0] = from_f<T>(v.x); O[1] = from_f<T>(v.y); O[2] = from_f<T>(v.z); O[3] = from_f<T>(v.w);
    return;
  }
  if (MODE != MODE_CONVT_FWD && splitk_vec<MODE>(g)) {
    // 4 consecutive columns per thread: 16-B partial loads, 4 splits' loads in flight, fixed split order
    const long long idx4 = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (idx4 >= total) return;
    const long long row = idx4 / g.Ncols;
    const int col = (int)(idx4 - row * g.Ncols);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    const float4* p = reinterpret_cast<const float4*>(g.part + idx4);
    const long long st = total / 4;
#pragma unroll 4
    for (int k = 0; k < g.ksplit; ++k) {
      const float4 a = p[(long long)k * st];
      v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
    }
    if (g.bias) {
      const float* bp = g.grp_n > 0 ? g.bias + (int)(row / ((long long)g.D * g.H * g.W) / g.grp_n) * g.b_gstride
                                    : g.bias;
      v.x += bp[col]; v.y += bp[col + 1]; v.z += bp[col + 2]; v.w += bp[col + 3];
    }
    T* O = out_at<T>(g, row, col);
    O[0] = from_f<T>(v.x); O[1] = from_f<T>(v.y); O[2] = from_f<T>(v.z); O[3] = from_f<T>(v.w);
    return;
  }
  long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const long long row = idx / g.Ncols;
  const int col = (int)(idx - row * g.Ncols);
  float v = 0.f;
  for (int k = 0; k < g.ksplit; ++k) v += g.part[(long long)k * total + idx];
  T* O = reinterpret_cast<T*>(g.out);
  if (MODE == MODE_CONVT_FWD) {
    const int Cout = g.Ncols >> 3;
    const int t = col / Cout, co = col - t * Cout;
    if (g.bias) v += g.bias[co];
    O[convt_child(row, t, g) * g.ldo + co] = from_f<T>(v);
  } else {
    if (g.bias)
      v += (g.grp_n > 0 ? g.bias + (int)(row / ((long long)g.D * g.H * g.W) / g.grp_n) * g.b_gstride : g.bias)[col];
    *out_at<T>(g, row, col) = from_f<T>(v);
  }
}

// Vectorised split-K reduce with the splits dealt over S slices of the block (256 / S float4 columns per
// block, ~4 splits per thread), slice sums a fixed pairwise LDS tree: at the small levels one thread per column
// walking 8..16 splits left the reduce latency-bound.  Same summation tree for every run (deterministic).
template <typename T, int S>
__global__ __launch_bounds__(256) void gemm_splitk_reduce_s(GemmArgs g) {
  constexpr int NC = 256 / S;
  __shared__ float4 red[S][NC];
  const long long total = (long long)g.M * g.Ncols;
  const int col4 = threadIdx.x % NC, sl = threadIdx.x / NC;
  const long long idx4 = ((long long)blockIdx.x * NC + col4) * 4;
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (idx4 < total) {
    const float4* p = reinterpret_cast<const float4*>(g.part + idx4);
    const long long st = total / 4;
#pragma unroll 4
    for (int k = sl; k < g.ksplit; k += S) {
      const float4 a = p[(long long)k * st];
      v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
    }
  }
  red[sl][col4] = v;
  __syncthreads();
#pragma unroll
  for (int h = S / 2; h > 0; h >>= 1) {
    if (sl < h) {
      const float4 a = red[sl + h][col4];
      v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
      red[sl][col4] = v;
    }
    __syncthreads();
  }
  if (sl != 0 || idx4 >= total) return;
  const long long row = idx4 / g.Ncols;
  const int col = (int)(idx4 - row * g.Ncols);
  if (g.bias) {
    const float* bp = g.grp_n > 0 ? g.bias + (int)(row / ((long long)g.D * g.H * g.W) / g.grp_n) * g.b_gstride
                                  : g.bias;
    v.x += bp[col]; v.y += bp[col + 1]; v.z += bp[col + 2]; v.w += bp[col + 3];
  }
  T* O = out_at<T>(g, row, col);
  O[0] = from_f<T>(v.x); O[1] = from_f<T>(v.y); O[2] = from_f<T>(v.z); O[3] = from_f<T>(v.w);
}

// ------------------------------------------------------------------ wgrad
// part[ks][row][col] = sum_{v in split ks} A[v][row] * Bgather[v][col]
//   CONV3 : A = dy (rows = Cout), B = x at v + off(tap), col = tap*Cin + ci
//   POINT : A = dy, B = x at v
//   CONVT : A = x (rows = Cin), B = dy at child(v, tap), col = tap*Cout + co
// Both operands are staged into LDS in their natural [voxel][channel] layout
// with 16-byte vector writes (double-buffered, one barrier per stage); the
// MFMA fragments (K = voxels) are read with the gfx950 transposed LDS read
// ds_read_b64_tr_b16 (bf16) or as single f32 elements (f32 path).
// bias_part (optional): the bias gradient partials.  A = dy (CONV3 / POINT): blocks of column tile 0 emit
// per-row sums of A, bias_part[ks][Ca].  CONVT: blocks of row tile 0 emit per-column sums of the gathered dy
// tile B, bias_part[ks][8 Cout] (col = tap*Cout + co), which mmseg_colsum_reduce folds over (ks, tap): the
// separate colsum pass over dy (113 MB at the 96^3 upconv) is not needed.
struct WgradArgs {
  const void* a;  int lda;
  const void* b;  int ldb;
  float* part;
  float* bias_part;
  int Ca, Ncols, cpg_shift;
  long long V;               // voxels in the a-grid
  int D, H, W;
  int ksplit;
  long long vox_per_split;   // multiple of KV
  int swz;
  int brick;                 // CONV3 only: ksplit splits the brick list instead of voxels
  // brick2 / brickr kernels (CONV3, bf16) write channel-major tiles (col = ci*27 + tap, the torch
  // order of grad[co][ci][3][3][3]); with ksplit == 1 and grad != null straight into the gradient.
  float* grad;
  float* bias_grad;
  int accumulate;
  int kchunks;               // CONV3 brick kernels: 32-channel chunks of x holding real channels (0 = all)
  // deferred InstanceNorm + ReLU of x (wgrad_brick2 only, mmseg_conv3_wgrad_norm): x holds the PRE-norm
  // activation, staged as relu((x - nmean[n][c]) * nrstd[n][c]) rounded to T
  const float* nmean;
  const float* nrstd;
  int dbg;   // brick weight-gradient timing probe (diagnostics builds): 1 = no global loads after the first brick, 2 = no MFMA
  int frag;  // wgrad_dma: split partials in the fragment-native layout (wgrad_dma_mt, WReduceArgs::frag_mt)
  int groups;  // grouped launch (wgrad_brickr only): the bricks are `groups` equal sample groups, splits
               // [gi * ksplit / groups, (gi + 1) * ksplit / groups) cover group gi's bricks only
  // grouped with one split per group (ksplit == groups) and grad != null: split gi writes group gi's gradient
  // straight to grad + gi * grad_gstride (bias_grad + gi * bias_gstride), no partials and no reduce
  long long grad_gstride;
  int bias_gstride;
  int grad_ld;   // direct gradient row pitch (27 x real input channels; 0 = Ncols), wgrad_direct_ok
  int pad16;   // mmseg_conv3_wgrad_ex phase bit 8: rows [Ca - 16, Ca) are output-channel padding (48 real of 64: the
               // SwinUNETR 48-channel levels); wgrad_dma's 64-co tile then runs 3 of its 4 MFMA row tiles, zero rows
};

// the launch writes the gradient itself: one split, or one split per group of a grouped launch
__device__ __forceinline__ bool wgrad_direct(const WgradArgs& g) {
  return g.ksplit == 1 || (g.groups > 1 && g.ksplit == g.groups);
}

__host__ __device__ __forceinline__ int wgrad_nchunk(int cpg_shift, int kchunks) {
  const int n = (8 << cpg_shift) / 32;
  return (kchunks > 0 && kchunks < n) ? kchunks : n;
}

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef short v8i16 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

__device__ __forceinline__ bf16x8 tr_frag(const bf16_t* p_lo, const bf16_t* p_hi) {
  v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(p_lo));
  v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(p_hi));
  v8i16 c = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, c);
}

template <int MODE>
__device__ __forceinline__ bool gather_src(long long vox, int kgi, int cpg_shift, const WgradArgs& g, long long& src,
                                           int& c8) {
  if (MODE == MODE_CONV3) {
    const int t = kgi >> cpg_shift;
    c8 = kgi & ((1 << cpg_shift) - 1);
    // 32-bit divisions (V < 2^31, checked by the host)
    const unsigned vu = (unsigned)vox;
    const unsigned q = vu / (unsigned)g.W, q2 = q / (unsigned)g.H;
    const int x = (int)(vu - q * (unsigned)g.W), y = (int)(q - q2 * (unsigned)g.H), z = (int)(q2 % (unsigned)g.D);
    int dz, dy, dx;
    tap_delta(t, dz, dy, dx);
    src = vox + ((long long)dz * g.H + dy) * g.W + dx;
    return (unsigned)(z + dz) < (unsigned)g.D && (unsigned)(y + dy) < (unsigned)g.H &&
           (unsigned)(x + dx) < (unsigned)g.W;
  } else if (MODE == MODE_CONVT_DGRAD) {
    const int t = kgi >> cpg_shift;
    c8 = kgi & ((1 << cpg_shift) - 1);
    const unsigned vu = (unsigned)vox;
    const unsigned q = vu / (unsigned)g.W, q2 = q / (unsigned)g.H, n = q2 / (unsigned)g.D;
    const unsigned x = vu - q * (unsigned)g.W, y = q - q2 * (unsigned)g.H, z = q2 - n * (unsigned)g.D;
    src = (((long long)n * 2LL * g.D + 2 * z + (t >> 2)) * 2LL * g.H + 2 * y + ((t >> 1) & 1)) * 2LL * g.W + 2 * x +
          (t & 1);
    return true;
  }
  c8 = kgi;
  src = vox;
  return true;
}

template <typename T, int MODE, int WM, int WN, int RM, int RN, int KV>
__global__ __launch_bounds__(256) void wgrad_kernel(WgradArgs g) {
  constexpr int BM = WM * RM * 16;
  constexpr int BN = WN * RN * 16;
  constexpr int EP = 16 / sizeof(T);
  constexpr int PA = BM + EP, PB = BN + EP;      // LDS row pitch (elements), 16-B aligned rows
  constexpr int AG = BM / 8, BG = BN / 8;
  constexpr int A_PER = KV * AG / 256, B_PER = KV * BG / 256;
  static_assert(A_PER >= 1 && B_PER >= 1 && (256 % AG) == 0 && (256 % BG) == 0, "tile/thread mismatch");
  constexpr int SA = KV * PA, SB = KV * PB;
  __shared__ __attribute__((aligned(16))) T lds[2 * (SA + SB)];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int ct_n = (g.Ncols + BN - 1) / BN, rt_n = (g.Ca + BM - 1) / BM;
  const int tile = g.swz ? xcd_swizzle(blockIdx.x, ct_n * rt_n * g.ksplit) : (int)blockIdx.x;
  const int ctile = tile % ct_n, rtile = (tile / ct_n) % rt_n, ks = tile / (ct_n * rt_n);
  const int row0 = rtile * BM;
  const int col0 = ctile * BN;
  const long long v_begin = ks * g.vox_per_split;
  long long v_end = v_begin + g.vox_per_split;
  if (v_end > g.V) v_end = g.V;
  const T* A = reinterpret_cast<const T*>(g.a);
  const T* B = reinterpret_cast<const T*>(g.b);
  constexpr bool BCOL = MODE == MODE_CONVT_DGRAD;   // bias = column sums of B (see above)
  const bool do_bias = g.bias_part != nullptr && (BCOL ? rtile == 0 : ctile == 0);

  // fixed per-thread column group (256 % BG == 0) -> fixed tap / channel group
  const int cga = tid % AG, cgb = tid % BG;
  const int kgi_b = (col0 >> 3) + cgb;
  const bool col_ok = kgi_b * 8 < g.Ncols;
  const bool row_ok = row0 + cga * 8 < g.Ca;

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float bsum[8] = {0, 0, 0, 0, 0, 0, 0, 0};

  V8<T> ra[A_PER], rb[B_PER];
  // transposed conv: the thread's B voxels step by KV per stage, so their (n, z, y, x) are decomposed once and
  // stepped (gather_src's three runtime divisions per load were ~29 VALU per MFMA, r04i PMC)
  int cx[B_PER], cy[B_PER], cz[B_PER], cn[B_PER];
  const int t_b = kgi_b >> g.cpg_shift, c8_b = kgi_b & ((1 << g.cpg_shift) - 1);
  if constexpr (MODE == MODE_CONVT_DGRAD) {
#pragma unroll
    for (int k = 0; k < B_PER; ++k) {
      const unsigned vu = (unsigned)(v_begin + (tid + k * 256) / BG);
      const unsigned q = vu / (unsigned)g.W, q2 = q / (unsigned)g.H;
      cn[k] = (int)(q2 / (unsigned)g.D);
      cz[k] = (int)(q2 - (unsigned)cn[k] * (unsigned)g.D);
      cy[k] = (int)(q - q2 * (unsigned)g.H);
      cx[k] = (int)(vu - q * (unsigned)g.W);
    }
  }
  auto load_stage = [&](long long vb) {
#pragma unroll
    for (int k = 0; k < A_PER; ++k) {
      const int v = (tid + k * 256) / AG;
      const long long vox = vb + v;
      if (vox < v_end && row_ok) ra[k].load(A + vox * g.lda + row0 + cga * 8);
      else ra[k].zero();
    }
#pragma unroll
    for (int k = 0; k < B_PER; ++k) {
      const int v = (tid + k * 256) / BG;
      const long long vox = vb + v;
      if constexpr (MODE == MODE_CONVT_DGRAD) {
        const unsigned src = (((unsigned)cn[k] * 2u * g.D + 2u * cz[k] + (t_b >> 2)) * 2u * g.H + 2u * cy[k] +
                              ((t_b >> 1) & 1)) * 2u * g.W + 2u * cx[k] + (t_b & 1);
        if (vox < v_end && col_ok) rb[k].load(B + (long long)src * g.ldb + c8_b * 8);
        else rb[k].zero();
        // step to the voxel KV further on (the next stage): one division for the x carry (KV may span several
        // rows of a small grid), then y / z wrap at most a few times
        cx[k] += KV;
        if (cx[k] >= g.W) {
          const int qy = (int)((unsigned)cx[k] / (unsigned)g.W);
          cx[k] -= qy * g.W;
          cy[k] += qy;
          while (cy[k] >= g.H) {
            cy[k] -= g.H;
            if (++cz[k] == g.D) {
              cz[k] = 0;
              ++cn[k];
            }
          }
        }
      } else {
        long long src;
        int c8;
        const bool ok = vox < v_end && col_ok && gather_src<MODE>(vox, kgi_b, g.cpg_shift, g, src, c8);
        if (ok) rb[k].load(B + src * g.ldb + c8 * 8);
        else rb[k].zero();
      }
    }
  };
  auto write_stage = [&](int buf) {
    T* As = lds + buf * (SA + SB);
    T* Bs = As + SA;
#pragma unroll
    for (int k = 0; k < A_PER; ++k) {
      const int v = (tid + k * 256) / AG;
      ra[k].store(As + v * PA + cga * 8);
      if (!BCOL && do_bias) {
#pragma unroll
        for (int j = 0; j < 8; ++j) bsum[j] += ra[k].get(j);
      }
    }
#pragma unroll
    for (int k = 0; k < B_PER; ++k) {
      const int v = (tid + k * 256) / BG;
      rb[k].store(Bs + v * PB + cgb * 8);
      if (BCOL && do_bias) {
#pragma unroll
        for (int j = 0; j < 8; ++j) bsum[j] += rb[k].get(j);
      }
    }
  };

  const int g4 = lane >> 4, i16 = lane & 15, q = i16 >> 2, p4 = i16 & 3;
  int buf = 0;
  if (v_begin < v_end) {
    load_stage(v_begin);
    write_stage(0);
  }
  __syncthreads();
  for (long long vb = v_begin; vb < v_end; vb += KV) {
    const bool more = vb + KV < v_end;
    if (more) load_stage(vb + KV);
    const T* As = lds + buf * (SA + SB);
    const T* Bs = As + SA;
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int kk = 0; kk < KV; kk += 32) {
        bf16x8 af[RM], bfr[RN];
#pragma unroll
        for (int i = 0; i < RM; ++i) {
          const bf16_t* base = (const bf16_t*)As + (kk + 8 * g4 + q) * PA + wm * RM * 16 + i * 16 + 4 * p4;
          af[i] = tr_frag(base, base + 4 * PA);
        }
#pragma unroll
        for (int j = 0; j < RN; ++j) {
          const bf16_t* base = (const bf16_t*)Bs + (kk + 8 * g4 + q) * PB + wn * RN * 16 + j * 16 + 4 * p4;
          bfr[j] = tr_frag(base, base + 4 * PB);
        }
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll 4
      for (int kk = 0; kk < KV; kk += 4) {
        float af[RM], bfr[RN];
#pragma unroll
        for (int i = 0; i < RM; ++i) af[i] = (float)As[(kk + g4) * PA + wm * RM * 16 + i * 16 + i16];
#pragma unroll
        for (int j = 0; j < RN; ++j) bfr[j] = (float)Bs[(kk + g4) * PB + wn * RN * 16 + j * 16 + i16];
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    if (more) write_stage(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }

#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      const int col = col0 + wn * RN * 16 + j * 16 + (lane & 15);
      if (col >= g.Ncols) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + wm * RM * 16 + i * 16 + (lane >> 4) * 4 + r;
        if (row >= g.Ca) continue;
        g.part[((long long)ks * g.Ca + row) * g.Ncols + col] = acc[i][j][r];
      }
    }
  if (do_bias) {
    // fixed-order reduction of the per-thread row (column) sums: threads with equal tid % AG (tid % BG) share
    // rows (columns)
    float* red = reinterpret_cast<float*>(lds);
#pragma unroll
    for (int j = 0; j < 8; ++j) red[tid * 8 + j] = bsum[j];
    __syncthreads();
    if (BCOL) {
      if (tid < BN) {
        const int cg = tid >> 3, j = tid & 7;
        float sacc = 0.f;
        for (int t = cg; t < 256; t += BG) sacc += red[t * 8 + j];
        if (col0 + tid < g.Ncols) g.bias_part[(long long)ks * g.Ncols + col0 + tid] = sacc;
      }
    } else if (tid < BM) {
      const int cg = tid >> 3, j = tid & 7;
      float sacc = 0.f;
      for (int t = cg; t < 256; t += AG) sacc += red[t * 8 + j];
      if (row0 + tid < g.Ca) g.bias_part[(long long)ks * g.Ca + row0 + tid] = sacc;
    }
  }
}

// ------------------------------------------------------- brick wgrad (3^3)
// dW[co][tap][ci] partials with the input halo reused by all 27 taps: a block
// owns 32 output channels x one 32-channel input chunk x ALL 27 taps, and walks
// a contiguous range of 4x4x8 bricks.  Per brick it stages dy [128 vox][32 co]
// and the x halo [6x6x10][32 ci] into LDS; K = the brick's 128 voxels.  The
// MFMA operands are read with ds_read_b64_tr_b16 (K = voxels is the strided
// dimension of NDHWC): the A rows come from the dy tile, the B rows from halo
// rows shifted by the tap (4 arbitrary row addresses per 16-lane group).
// Wave w accumulates taps [7w, 7w+7) -> 2 x 7 x 2 MFMA tiles in registers.
template <typename T>
__global__ __launch_bounds__(256) void wgrad_brick_kernel(WgradArgs g) {
  constexpr int EP = 16 / sizeof(T);
  constexpr int DP = 32 + EP;                    // dy tile pitch
  constexpr int XP = CK + EP;                    // halo pitch
  constexpr int DS = 128 * DP, XS = HLO_V * XP;
  __shared__ __attribute__((aligned(16))) T lds[DS + XS];
  T* Dl = lds;
  T* Xl = lds + DS;
  constexpr int D_ITEMS = 128 * 4, X_ITEMS = HLO_V * 4;
  constexpr int D_PER = D_ITEMS / 256, X_PER = (X_ITEMS + 255) / 256;

  const T* Dy = reinterpret_cast<const T*>(g.a);
  const T* X = reinterpret_cast<const T*>(g.b);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cin = 8 << g.cpg_shift;
  const int nchunk = wgrad_nchunk(g.cpg_shift, g.kchunks), rt_n = g.Ca / 32;
  const int tile = blockIdx.x;
  const int ct = tile % nchunk, rt = (tile / nchunk) % rt_n, ks = tile / (nchunk * rt_n);
  const int bz_n = g.D / BRK_Z, by_n = g.H / BRK_Y, bx_n = g.W / BRK_X;
  const long long nbrick = (g.V / ((long long)g.D * g.H * g.W)) * bz_n * by_n * bx_n;
  const long long bpk = (nbrick + g.ksplit - 1) / g.ksplit;
  const long long b_begin = ks * bpk;
  const long long b_end = b_begin + bpk < nbrick ? b_begin + bpk : nbrick;
  const long long HW = (long long)g.H * g.W;
  const int row0 = rt * 32, c0 = ct * CK;
  const bool do_bias = g.bias_part != nullptr && ct == 0;
  const int t_begin = wave * 7, t_cnt = wave == 3 ? 6 : 7;

  f32x4 acc[2][7][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int t = 0; t < 7; ++t)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][t][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float bsum[8] = {0, 0, 0, 0, 0, 0, 0, 0};

  V8<T> dr[D_PER], xr[X_PER];
  auto brick_origin = [&](long long b, long long& nbase, int& z0, int& y0, int& x0) {
    int q = (int)b;   // brick index < V / 128 < 2^31 (mmseg_wgrad): 32-bit division
    const int bx = q % bx_n;
    q /= bx_n;
    const int by = q % by_n;
    q /= by_n;
    const int bz = q % bz_n;
    const long long n = q / bz_n;
    nbase = n * g.D * HW;
    z0 = bz * BRK_Z;
    y0 = by * BRK_Y;
    x0 = bx * BRK_X;
  };
  auto load = [&](long long b) {
    long long nbase;
    int z0, y0, x0;
    brick_origin(b, nbase, z0, y0, x0);
#pragma unroll
    for (int k = 0; k < D_PER; ++k) {
      const int e = tid + k * 256, v = e >> 2, cg = e & 3;
      const int z = z0 + (v >> 5), y = y0 + ((v >> 3) & 3), x = x0 + (v & 7);
      dr[k].load(Dy + (nbase + z * HW + (long long)y * g.W + x) * g.lda + row0 + cg * 8);
    }
#pragma unroll
    for (int k = 0; k < X_PER; ++k) {
      const int e = tid + k * 256;
      if (e < X_ITEMS) {
        const int h = e >> 2, cg = e & 3;
        const int hx = h % HLO_X, hy = (h / HLO_X) % HLO_Y, hz = h / (HLO_X * HLO_Y);
        const int z = z0 - 1 + hz, y = y0 - 1 + hy, x = x0 - 1 + hx;
        if ((unsigned)z < (unsigned)g.D && (unsigned)y < (unsigned)g.H && (unsigned)x < (unsigned)g.W)
          xr[k].load(X + (nbase + z * HW + (long long)y * g.W + x) * g.ldb + c0 + cg * 8);
        else
          xr[k].zero();
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int k = 0; k < D_PER; ++k) {
      const int e = tid + k * 256;
      dr[k].store(Dl + (e >> 2) * DP + (e & 3) * 8);
      if (do_bias) {
#pragma unroll
        for (int j = 0; j < 8; ++j) bsum[j] += dr[k].get(j);
      }
    }
#pragma unroll
    for (int k = 0; k < X_PER; ++k) {
      const int e = tid + k * 256;
      if (e < X_ITEMS) xr[k].store(Xl + (e >> 2) * XP + (e & 3) * 8);
    }
  };

  const int g4 = lane >> 4, i16 = lane & 15, q = i16 >> 2, p4 = i16 & 3;
  if (b_begin < b_end) {
    load(b_begin);
    store();
  }
  __syncthreads();
  for (long long b = b_begin; b < b_end; ++b) {
    const bool more = b + 1 < b_end;
    if (more) load(b + 1);
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int kk = 0; kk < 128; kk += 32) {
        bf16x8 af[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const bf16_t* base = (const bf16_t*)Dl + (kk + 8 * g4 + q) * DP + i * 16 + 4 * p4;
          af[i] = tr_frag(base, base + 4 * DP);
        }
        // B rows: voxels v = kk + 8*g4 + q (+4) -> halo row of (v) shifted by the tap
        const int v_lo = kk + 8 * g4 + q, v_hi = v_lo + 4;
        const int hlo = ((v_lo >> 5) * HLO_Y + ((v_lo >> 3) & 3)) * HLO_X + (v_lo & 7);
        const int hhi = ((v_hi >> 5) * HLO_Y + ((v_hi >> 3) & 3)) * HLO_X + (v_hi & 7);
#pragma unroll
        for (int t = 0; t < 7; ++t) {
          if (t < t_cnt) {
            const int tap = t_begin + t;
            const int kz = tap / 9, ky = (tap / 3) % 3, kx = tap % 3;
            const int hoff = (kz * HLO_Y + ky) * HLO_X + kx;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const bf16_t* pl = (const bf16_t*)Xl + (hlo + hoff) * XP + j * 16 + 4 * p4;
              const bf16_t* ph = (const bf16_t*)Xl + (hhi + hoff) * XP + j * 16 + 4 * p4;
              const bf16x8 bfr = tr_frag(pl, ph);
#pragma unroll
              for (int i = 0; i < 2; ++i)
                acc[i][t][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr, acc[i][t][j], 0, 0, 0);
            }
          }
        }
      }
    } else {
      for (int kk = 0; kk < 128; kk += 4) {
        const int v = kk + g4;
        const int hv = ((v >> 5) * HLO_Y + ((v >> 3) & 3)) * HLO_X + (v & 7);
        float af[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) af[i] = (float)Dl[v * DP + i * 16 + i16];
#pragma unroll
        for (int t = 0; t < 7; ++t) {
          if (t < t_cnt) {
            const int tap = t_begin + t;
            const int kz = tap / 9, ky = (tap / 3) % 3, kx = tap % 3;
            const int hoff = (kz * HLO_Y + ky) * HLO_X + kx;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const float bv = (float)Xl[(hv + hoff) * XP + j * 16 + i16];
#pragma unroll
              for (int i = 0; i < 2; ++i)
                acc[i][t][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bv, acc[i][t][j], 0, 0, 0);
            }
          }
        }
      }
    }
    __syncthreads();
    if (more) {
      store();
      __syncthreads();
    }
  }

  // partial layout [ks][Ca][Ncols], col = tap*cin + ci
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int t = 0; t < 7; ++t) {
      if (t >= t_cnt) continue;
      const int tap = t_begin + t;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = tap * cin + c0 + j * 16 + i16;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = row0 + i * 16 + g4 * 4 + r;
          g.part[((long long)ks * g.Ca + row) * g.Ncols + col] = acc[i][t][j][r];
        }
      }
    }
  if (do_bias) {
    float* red = reinterpret_cast<float*>(lds);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j) red[tid * 8 + j] = bsum[j];
    __syncthreads();
    if (tid < 32) {
      const int cg = tid >> 3, j = tid & 7;
      float sacc = 0.f;
      for (int t = cg; t < 256; t += 4) sacc += red[t * 8 + j];
      g.bias_part[(long long)ks * g.Ca + row0 + tid] = sacc;
    }
  }
}


// Epilogue of the brick wgrad kernels (8 waves, acc[t][i][j] = rows i*16.., input channels j*16.., tap
// t_begin + t): the block's [MT*16 co][32 ci][27 taps] fp32 tile goes through LDS 16 co-rows at a time and
// leaves as contiguous float4 rows in channel-major order (torch grad[co][ci][tap] order), either into the
// split partial part[ks][Ca][Ncols] or, for a single split, straight into the gradient (= or +=).
// LDS pitch 868 floats: a ds_write_b32 lane group (two co-rows x 16 ci, ci stride 27) hits 32 distinct banks.
constexpr int WEP_P = 868;
// RP rows of the 16-row MFMA tile per LDS pass (16: 55.5 KB of staging; 8: half that, two passes)
template <int MT, int RP = 16>
__device__ __forceinline__ void wgrad_store_chmajor(const f32x4 (&acc)[4][MT][2], int t_begin, int t_cnt, float* L,
                                                    const WgradArgs& g, int ks, int row0, int c0) {
  const int tid = threadIdx.x, lane = tid & 63, g4 = lane >> 4, i16 = lane & 15;
  const bool direct = g.grad != nullptr && wgrad_direct(g);
  float* base = direct ? g.grad + (g.ksplit > 1 ? (long long)ks * g.grad_gstride : 0LL)
                       : g.part + (long long)ks * g.Ca * g.Ncols;
  const long long ldg = direct && g.grad_ld > 0 ? g.grad_ld : g.Ncols;   // gradient row pitch (real channels)
  const bool accum = direct && g.accumulate;
  constexpr int GP = RP / 4;   // lane groups per pass
#pragma unroll
  for (int i = 0; i < MT; ++i) {
#pragma unroll
    for (int hh = 0; hh < 16 / RP; ++hh) {
      __syncthreads();
      if (g4 / GP == hh) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          if (t >= t_cnt) continue;
          const int tap = t_begin + t;
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) L[((g4 % GP) * 4 + r) * WEP_P + (j * 16 + i16) * 27 + tap] = acc[t][i][j][r];
        }
      }
      __syncthreads();
      for (int e = tid; e < RP * 216; e += 512) {
        const int rr = e / 216, q = e - rr * 216;
        const float4 v = *reinterpret_cast<const float4*>(L + rr * WEP_P + q * 4);
        float4* d = reinterpret_cast<float4*>(base + (long long)(row0 + i * 16 + hh * RP + rr) * ldg + c0 * 27 +
                                              q * 4);
        if (accum) {
          const float4 o = *d;
          *d = make_float4(o.x + v.x, o.y + v.y, o.z + v.z, o.w + v.w);
        } else {
          *d = v;
        }
      }
    }
  }
}

template <int CG>
__device__ __forceinline__ void wgrad_store_bias(const float (&bsum)[8], float* red, const WgradArgs& g, int ks,
                                                 int row0) {
  constexpr int CO = CG * 8;
  const int tid = threadIdx.x;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 8; ++j) red[tid * 8 + j] = bsum[j];
  __syncthreads();
  if (tid < CO) {
    const int cg = tid >> 3, j = tid & 7;
    float sacc = 0.f;
    for (int t = cg; t < 512; t += CG) sacc += red[t * 8 + j];
    if (g.bias_grad != nullptr && wgrad_direct(g)) {
      float* bg = g.bias_grad + (g.ksplit > 1 ? ks * g.bias_gstride : 0) + row0 + tid;
      *bg = g.accumulate ? *bg + sacc : sacc;
    } else {
      g.bias_part[(long long)ks * g.Ca + row0 + tid] = sacc;
    }
  }
}

// ------------------------------------------------ brick wgrad v2 (3^3)
// 8 waves, 64 output channels x one 32-channel input chunk x all 27 taps per
// block (wgrad_brick_kernel has 32 x 32): each tap-shifted halo fragment now
// feeds 4 MFMAs instead of 2 and one staged halo serves twice the output
// channels, so LDS reads and L2 traffic per MAC drop by a third.  Taps are
// dealt 4,4,4,3,3,3,3,3 over the waves (acc: 4 taps x 4 x 2 tiles = 128
// VGPRs).  The two LDS stage buffers alternate, one barrier per brick.
// V = 3 (default): bank-conflict-free transposed reads.  A ds_read_b64_tr_b16 half-wave reads 8 tile rows
// x 16 columns; with the K order below those 8 rows are 8 consecutive voxels (one x-row of the brick: lane
// group g4, element j -> x = 4*(g4&1) + (j&3), y = 2*(g4>>1) + (j>>2)) in BOTH the dy tile and the halo, and
// with row pitches of 24 or 40 dwords (== 8 mod 16) 8 consecutive rows cover the 64 banks exactly once.
// V = 2: the previous K order (x = j&3 + 4*(j>>2), y = g4) with 20-dword pitches, 2-way conflicted
// (SQ_LDS_BANK_CONFLICT = half the LDS-active cycles at 96^3).
// NORM: x holds a pre-norm activation (g.nmean / g.nrstd, mmseg_conv3_wgrad_norm); a separate instantiation so
// the plain kernel does not carry the statistics' registers (256 VGPRs + spills for CO64 otherwise)
// PIPE (bf16, V = 3): the software-pipelined multiply of wgrad_dma_kernel's PIPE form -- halo fragments two
// (dy plane, tap) steps ahead in a ring of three, dy fragments one plane ahead -- instead of reading each tap's
// fragments into the registers the previous tap's MFMAs just released (read, wait, 4 MFMAs, per tap).
template <typename T, int MT, int V, bool NORM = false, bool PIPE = false>
__global__ __launch_bounds__(512, (MT == 2 && V == 2) ? 2 : 1) void wgrad_brick2_kernel(WgradArgs g) {
  static_assert(!PIPE || (V == 3 && sizeof(T) == 2), "PIPE: bf16 with the V = 3 fragment order");
  constexpr int EP = 16 / sizeof(T);
  constexpr int CO = MT * 16, CG = CO / 8;       // output channels per block, 8-channel groups
  constexpr int DP = V == 3 ? (MT == 2 ? 48 : 80) : CO + EP;   // dy tile pitch (elements)
  constexpr int XP = V == 3 ? 48 : CK + EP;                    // halo pitch
  constexpr int DS = 128 * DP, XS = HLO_V * XP;
  __shared__ __attribute__((aligned(16))) T lds[2 * (DS + XS)];
  constexpr int D_ITEMS = 128 * CG, X_ITEMS = HLO_V * 4;
  constexpr int D_PER = D_ITEMS / 512, X_PER = (X_ITEMS + 511) / 512;

  const T* Dy = reinterpret_cast<const T*>(g.a);
  const T* X = reinterpret_cast<const T*>(g.b);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cin = 8 << g.cpg_shift;
  const int nchunk = wgrad_nchunk(g.cpg_shift, g.kchunks), rt_n = g.Ca / CO;
  const int tile = g.swz ? xcd_swizzle(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int ct = tile % nchunk, rt = (tile / nchunk) % rt_n, ks = tile / (nchunk * rt_n);
  const int bz_n = g.D / BRK_Z, by_n = g.H / BRK_Y, bx_n = g.W / BRK_X;
  const long long nbrick = (g.V / ((long long)g.D * g.H * g.W)) * bz_n * by_n * bx_n;
  const long long bpk = (nbrick + g.ksplit - 1) / g.ksplit;
  const long long b_begin = ks * bpk;
  const long long b_end = b_begin + bpk < nbrick ? b_begin + bpk : nbrick;
  const long long HW = (long long)g.H * g.W;
  const int row0 = rt * CO, c0 = ct * CK;
  const bool do_bias = g.bias_part != nullptr && ct == 0;
  // wave-uniform (SGPRs): the per-tap halo offsets are scalar, and the pipelined multiply branches on t_cnt
  const int t_begin = __builtin_amdgcn_readfirstlane(wave < 3 ? 4 * wave : 12 + 3 * (wave - 3));
  const int t_cnt = __builtin_amdgcn_readfirstlane(wave < 3 ? 4 : 3);

  f32x4 acc[4][MT][2];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[t][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float bsum[8] = {0, 0, 0, 0, 0, 0, 0, 0};

  V8<T> dr[D_PER], xr[X_PER];
  uint32_t xin = 0;    // bit k: xr[k] is an in-volume voxel (padding stays 0 under the deferred norm)
  int xn = 0;          // sample of the staged brick
  int norm_n = -1;     // sample whose deferred-norm statistics nmu / nrs hold
  float nmu[NORM ? 8 : 1], nrs[NORM ? 8 : 1];
  auto load_into = [&](long long b, auto& dr, auto& xr, uint32_t& xin, int& xn) {
    int q = (int)b;   // brick index < V / 128 < 2^31 (mmseg_wgrad): 32-bit division
    const int bx = q % bx_n;
    q /= bx_n;
    const int by = q % by_n;
    q /= by_n;
    const int bz = q % bz_n;
    xn = q / bz_n;
    const long long nbase = (long long)xn * g.D * HW;
    const int z0 = bz * BRK_Z, y0 = by * BRK_Y, x0 = bx * BRK_X;
    xin = 0;
#pragma unroll
    for (int k = 0; k < D_PER; ++k) {
      const int e = tid + k * 512, v = e / CG, cg = e % CG;
      const int z = z0 + (v >> 5), y = y0 + ((v >> 3) & 3), x = x0 + (v & 7);
      dr[k].load(Dy + (nbase + z * HW + (long long)y * g.W + x) * g.lda + row0 + cg * 8);
    }
#pragma unroll
    for (int k = 0; k < X_PER; ++k) {
      const int e = tid + k * 512;
      if (e < X_ITEMS) {
        const int h = e >> 2, cg = e & 3;
        const int hx = h % HLO_X, hy = (h / HLO_X) % HLO_Y, hz = h / (HLO_X * HLO_Y);
        const int z = z0 - 1 + hz, y = y0 - 1 + hy, x = x0 - 1 + hx;
        if ((unsigned)z < (unsigned)g.D && (unsigned)y < (unsigned)g.H && (unsigned)x < (unsigned)g.W) {
          xr[k].load(X + (nbase + z * HW + (long long)y * g.W + x) * g.ldb + c0 + cg * 8);
          if constexpr (NORM) xin |= 1u << k;
        } else {
          xr[k].zero();
        }
      }
    }
  };
  auto store_from = [&](int buf, auto& dr, auto& xr, uint32_t xin, int xn) {
    T* Dl = lds + buf * (DS + XS);
    T* Xl = Dl + DS;
#pragma unroll
    for (int k = 0; k < D_PER; ++k) {
      const int e = tid + k * 512;
      dr[k].store(Dl + (e / CG) * DP + (e % CG) * 8);
      if (do_bias) {
#pragma unroll
        for (int j = 0; j < 8; ++j) bsum[j] += dr[k].get(j);
      }
    }
    if constexpr (NORM) {   // deferred InstanceNorm + ReLU of x: channels c0 + 8 (tid & 3) .. of sample xn
      if (xn != norm_n) {   // (the statistics change only when the brick range crosses into the next sample)
        norm_n = xn;
        const int cb = xn * cin + c0 + (tid & 3) * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          nmu[j] = g.nmean[cb + j];
          nrs[j] = g.nrstd[cb + j];
        }
      }
#pragma unroll
      for (int k = 0; k < X_PER; ++k)
        if ((xin >> k) & 1u) norm_relu8<T>(xr[k], nmu, nrs);
    }
#pragma unroll
    for (int k = 0; k < X_PER; ++k) {
      const int e = tid + k * 512;
      if (e < X_ITEMS) xr[k].store(Xl + (e >> 2) * XP + (e & 3) * 8);
    }
  };

  const int g4 = lane >> 4, i16 = lane & 15, q = i16 >> 2, p4 = i16 & 3;
  auto compute = [&](int buf) {
    const T* Dl = lds + buf * (DS + XS);
    const T* Xl = Dl + DS;
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int kk = 0; kk < 128; kk += 32) {
        bf16x8 af[MT];
        const int v_lo = V == 3 ? kk + 16 * (g4 >> 1) + 4 * (g4 & 1) + q : kk + 8 * g4 + q;
        const int v_hi = V == 3 ? v_lo + 8 : v_lo + 4;
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          const bf16_t* base = (const bf16_t*)Dl + v_lo * DP + i * 16 + 4 * p4;
          af[i] = tr_frag(base, base + (v_hi - v_lo) * DP);
        }
        const int hlo = ((v_lo >> 5) * HLO_Y + ((v_lo >> 3) & 3)) * HLO_X + (v_lo & 7);
        const int hhi = ((v_hi >> 5) * HLO_Y + ((v_hi >> 3) & 3)) * HLO_X + (v_hi & 7);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          if (t < t_cnt) {
            const int tap = t_begin + t;
            const int kz = tap / 9, ky = (tap / 3) % 3, kx = tap % 3;
            const int hoff = (kz * HLO_Y + ky) * HLO_X + kx;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const bf16_t* pl = (const bf16_t*)Xl + (hlo + hoff) * XP + j * 16 + 4 * p4;
              const bf16_t* ph = (const bf16_t*)Xl + (hhi + hoff) * XP + j * 16 + 4 * p4;
              const bf16x8 bfr = tr_frag(pl, ph);
#pragma unroll
              for (int i = 0; i < MT; ++i)
                acc[t][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr, acc[t][i][j], 0, 0, 0);
            }
          }
        }
      }
    } else {
      for (int kk = 0; kk < 128; kk += 4) {
        const int v = kk + g4;
        const int hv = ((v >> 5) * HLO_Y + ((v >> 3) & 3)) * HLO_X + (v & 7);
        float af[MT];
#pragma unroll
        for (int i = 0; i < MT; ++i) af[i] = (float)Dl[v * DP + i * 16 + i16];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          if (t < t_cnt) {
            const int tap = t_begin + t;
            const int kz = tap / 9, ky = (tap / 3) % 3, kx = tap % 3;
            const int hoff = (kz * HLO_Y + ky) * HLO_X + kx;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const float bv = (float)Xl[(hv + hoff) * XP + j * 16 + i16];
#pragma unroll
              for (int i = 0; i < MT; ++i)
                acc[t][i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bv, acc[t][i][j], 0, 0, 0);
            }
          }
        }
      }
    }
  };

  // PIPE: steps s = (dy plane k4, tap t) over this wave's TC taps; lane rows v_lo = 32 k4 + v0 and v_lo + 8 (halo
  // rows hlo and hlo + HLO_X of the tap's shifted window)
  const int v0 = 16 * (g4 >> 1) + 4 * (g4 & 1) + q;
  const int hlo0 = ((v0 >> 3) & 3) * HLO_X + (v0 & 7);
  auto compute_pipe = [&](int buf, auto tcc) __attribute__((always_inline)) {
    if constexpr (PIPE) {
      constexpr int TC = decltype(tcc)::value;
      constexpr int PD = 3, NS = 4 * TC;
      const bf16_t* Dl = reinterpret_cast<const bf16_t*>(lds + buf * (DS + XS));
      const bf16_t* Xl = Dl + DS;
      bf16x8 af[2][MT], bf[PD][2];
      auto load_a = [&](int k4, bf16x8(&a)[MT]) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          const bf16_t* base = Dl + (32 * k4 + v0) * DP + i * 16 + 4 * p4;
          a[i] = tr_frag(base, base + 8 * DP);
        }
      };
      auto load_b = [&](int k4, int t, bf16x8(&b)[2]) __attribute__((always_inline)) {
        const int tap = t_begin + t;
        const int kz = tap / 9, ky = (tap / 3) % 3, kx = tap % 3;
        const int h = k4 * (HLO_Y * HLO_X) + hlo0 + (kz * HLO_Y + ky) * HLO_X + kx;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const bf16_t* pl = Xl + h * XP + j * 16 + 4 * p4;
          b[j] = tr_frag(pl, pl + HLO_X * XP);
        }
      };
      load_a(0, af[0]);
#pragma unroll
      for (int s0 = 0; s0 < PD - 1; ++s0)
        if (s0 < NS) load_b(s0 / TC, s0 % TC, bf[s0 % PD]);
#pragma unroll
      for (int sidx = 0; sidx < NS; ++sidx) {
        const int k4 = sidx / TC, t = sidx % TC;
        const int sn = sidx + PD - 1;
        if (sn < NS) load_b(sn / TC, sn % TC, bf[sn % PD]);
        if (t == 0 && k4 + 1 < 4) load_a(k4 + 1, af[(k4 + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int i = 0; i < MT; ++i)
            acc[t][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[k4 & 1][i], bf[sidx % PD][j], acc[t][i][j], 0,
                                                                   0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };

  // PIPE: the brick loop is instantiated per tap count (a branch inside it would merge the two multiplies'
  // accumulator registers at every brick: copies, and 256 VGPRs with spills)
  auto brick_loop = [&](auto tcc) __attribute__((always_inline)) {
    int buf = 0;
    if (b_begin < b_end) {
      load_into(b_begin, dr, xr, xin, xn);
      store_from(0, dr, xr, xin, xn);
    }
    __syncthreads();
    for (long long b = b_begin; b < b_end; ++b) {
      const bool more = b + 1 < b_end;
      if (more && g.dbg != 1) load_into(b + 1, dr, xr, xin, xn);
      if (g.dbg != 2) {
        if constexpr (PIPE)
          compute_pipe(buf, tcc);
        else
          compute(buf);
      }
      if (more) store_from(buf ^ 1, dr, xr, xin, xn);
      __syncthreads();
      buf ^= 1;
    }
  };
  if (!PIPE || t_cnt == 4)
    brick_loop(std::integral_constant<int, 4>{});
  else
    brick_loop(std::integral_constant<int, 3>{});

  static_assert(sizeof(lds) >= 16 * WEP_P * sizeof(float) && sizeof(lds) >= 512 * 8 * sizeof(float),
                "epilogue staging must fit the stage buffers");
  wgrad_store_chmajor<MT>(acc, t_begin, t_cnt, reinterpret_cast<float*>(lds), g, ks, row0, c0);
  if (do_bias) wgrad_store_bias<CG>(bsum, reinterpret_cast<float*>(lds), g, ks, row0);
}

// ------------------------------------------ brick wgrad, LDS-DMA staging (3^3, bf16)
// wgrad_brick2_kernel<bf16, MT, 3> with the stage images filled by buffer_load ... lds (no staging registers,
// no ds_write) into THREE stage buffers: brick b + 2 is in flight while brick b is multiplied, so a load has two
// brick periods to land instead of one (the register-staged kernel spends about a third of its time waiting
// on its one-brick-ahead loads: 136 us with, 105 us without loads at 96^3 32->32).  The rows are unpadded and
// XOR-swizzled at 32-byte granules instead (the DMA writes 64 contiguous 16-B chunks per wave-instruction; the
// lane picks the global chunk that belongs at its LDS position), which keeps the transposed fragment reads
// conflict-free:
//   halo row (hz, hy, hx), 64 B:   granule j of channel half j lives at j ^ ((hx >> 2) & 1)
//   dy row v, 64 B (32 co):        granule i at i ^ ((v >> 2) & 1)
//   dy row v, 128 B (64 co):       granule i at i ^ ((v >> 1) & 3)
// (8 consecutive halo x positions, or 8 aligned dy rows, then cover the 64 banks once).  The bias gradient
// is one more MFMA chain against a ones fragment in wave 7's free tap slot.  NORM: the deferred InstanceNorm +
// ReLU is applied in place to the landed halo (each thread its fixed channel group), one extra barrier.
// (WD_OOB, wd_rsrc, wd_dma16: mmseg_common.h)

// ------------------------------------------------- brick conv v8 (3^3, bf16, 8 waves, LDS-DMA staging)
// conv3_brick2's BN-column tile with the block grown to an (8 ZP) x 8 x 8 brick: 8 waves, wave w owns z planes
// w ZP .. w ZP + ZP - 1 (64 voxels each = 4 row tiles of two 8-voxel x rows) x BN columns (BN 64 with ZP 1; BN 32
// with ZP 2, so a wave still runs 16 MFMAs per tap).  Both operands are staged by LDS-DMA
// (buffer_load ... lds): no staging registers and no ds_write pass, which in conv3_brick2 were ~2 VALU + 0.7 SALU
// per MFMA around a per-stage register round trip of the weights.  Per block:
//   * the halo image of one 32-channel input chunk: 10 x 10 rows of 10 voxels x 4 quads + 2 pad quads (the pad
//     keeps the 16-lane groups of the A-fragment ds_read_b128 on distinct banks), single buffer, re-filled
//     between chunks (that refill is the one exposed load: 1 of 3 * nchunk stages);
//   * the weight slice of one (chunk, kz) stage: 9 taps x BN columns x 32 channels in the B-operand order
//     [tap][col][4 quads, channel group kg at slot kg ^ w2_swz(col)], double buffered: stage s + 1's slice
//     lands while stage s is multiplied.
// The lane-linear DMA destination is matched by computing, per lane, the source of the quad that belongs at its
// LDS slot (pads and out-of-volume voxels read zeros through the OOB offset).  Each staged weight slice feeds
// 8 waves x 9 taps x 4 ZP x RN MFMAs (twice conv3_brick2's).  LDS 141 KB (BN 64) / 155 KB (BN 32): one block per
// CU, two waves per SIMD.  Requirements (host): bf16, Cin % 32 == 0, Ncols % BN == 0, D % 8 ZP, H % 8, W % 8, ksplit == 1, no
// fused stats / deferred norm / IN partials, the A and B extents < 2^31 bytes.
template <int BN, int ZP>
__global__ __launch_bounds__(512, 1) void conv3_brick8_kernel(GemmArgs g) {
  PROBE_BLOCK(false);
  PROBE_DECL();
  typedef bf16_t T;
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  constexpr int QV = 4;                                  // 16-B quads per halo voxel (32 channels)
  constexpr int BZ = 8 * ZP;                            // z planes per brick (ZP per wave)
  constexpr int HXY = 10, HZ = BZ + 2;
  constexpr int RY = HXY * QV + 2, RZ = HXY * RY;        // 42 quads per halo row, 420 per plane
  constexpr int XQ = HZ * RZ;                            // 4200 (ZP 1) / 7560 (ZP 2)
  constexpr int XI = (XQ + 63) / 64, XK = (XI + 7) / 8;  // 66 / 119 wave-instructions
  constexpr int XQP = XI * 64;
  constexpr int WQ = 9 * BN * QV;                        // 2304 quads (BN 64)
  constexpr int WI = WQ / 64, WK = (WI + 7) / 8;         // 36, <= 5 per wave
  constexpr int RM = 4 * ZP, RN = BN / 16;
  constexpr int EPQ = 8;                                 // bf16 per quad
  static_assert(WQ % 64 == 0, "weight slice must be whole wave-instructions");
  __shared__ __attribute__((aligned(16))) float4 lds4[XQP + 2 * WQ];
  T* Xl = reinterpret_cast<T*>(lds4);
  T* Wl = reinterpret_cast<T*>(lds4 + XQP);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bz_n = g.D / BZ, by_n = g.H >> 3, bx_n = g.W >> 3;
  const int nbrick = (g.M / (g.D * g.H * g.W)) * bz_n * by_n * bx_n;
  const int nt_n = g.Ncols / BN;
  const int tile = g.swz ? xcd_swizzle(blockIdx.x, nbrick * nt_n) : (int)blockIdx.x;
  int bidx = tile % nbrick;
  const int nt = tile / nbrick;
  const int bx = bidx % bx_n; bidx /= bx_n;
  const int by = bidx % by_n; bidx /= by_n;
  const int bz = bidx % bz_n;
  const int n = bidx / bz_n;
  const int z0 = bz * BZ, y0 = by * 8, x0 = bx * 8;
  const int n0 = nt * BN;
  const int cin = 8 << g.cpg_shift;
  const int nchunk = gemm_nchunk(g);
  const int nstage = nchunk * 3;
  const long long HW = (long long)g.H * g.W;
  const long long nbase = (long long)n * g.D * HW;

  const wd_rsrc_t arsrc = wd_rsrc(g.a, (uint32_t)((long long)g.M * g.lda * 2));
  const int KGp = (g.KG + 3) & ~3;
  const wd_rsrc_t brsrc = wd_rsrc(g.b, (uint32_t)((long long)KGp * g.Cpad * 16));

  // per-lane halo sources: quad p = 64 m + lane of instruction m = wave + 8 kk, byte offset of chunk 0 or OOB
  uint32_t xo[XK];
#pragma unroll
  for (int kk = 0; kk < XK; ++kk) {
    const int p = (wave + 8 * kk) * 64 + lane;
    const int row = p / RY, qi = p - row * RY;
    const int hz = row / HXY, hy = row - hz * HXY, hx = qi >> 2, cg = qi & 3;
    const int z = z0 - 1 + hz, y = y0 - 1 + hy, x = x0 - 1 + hx;
    const bool ok = p < XQ && qi < HXY * QV && (unsigned)z < (unsigned)g.D && (unsigned)y < (unsigned)g.H &&
                    (unsigned)x < (unsigned)g.W;
    xo[kk] = ok ? (uint32_t)((((n * g.D + z) * g.H + y) * g.W + x) * g.lda * 2 + cg * 16) : WD_OOB;
  }
  // per-lane weight sources: quad p = (t9 * BN + col) * 4 + slot, channel group slot ^ w2_swz(col)
  uint32_t wo[WK];
#pragma unroll
  for (int kk = 0; kk < WK; ++kk) {
    const int p = (wave + 8 * kk) * 64 + lane;
    const int q = p >> 2, col = q % BN, t9 = q / BN;
    const int cg = (p & 3) ^ w2_swz(col);
    wo[kk] = (uint32_t)(((t9 * (cin / 8) + cg) * g.Cpad + n0 + col) * 16);
  }
  const uint32_t xl_base = (uint32_t)(uintptr_t)(lds_ptr_t)Xl;
  const uint32_t wl_base = (uint32_t)(uintptr_t)(lds_ptr_t)Wl;
  auto issue_x = [&](int c) {
#pragma unroll
    for (int kk = 0; kk < XK; ++kk) {
      const int m = wave + 8 * kk;
      if (m < XI)
        wd_dma16(__builtin_amdgcn_readfirstlane((int)(xl_base + m * 1024)),
                 xo[kk] == WD_OOB ? WD_OOB : xo[kk] + c * 64, arsrc);
    }
  };
  auto issue_w = [&](int s, int buf) {
    const int c = s / 3, kz = s - c * 3;
    const uint32_t so = (uint32_t)((kz * 9 * (cin / 8) + c * 4) * g.Cpad * 16);
#pragma unroll
    for (int kk = 0; kk < WK; ++kk) {
      const int m = wave + 8 * kk;
      if (m < WI)
        wd_dma16(__builtin_amdgcn_readfirstlane((int)(wl_base + (buf * WQ + m * 64) * 16)), wo[kk] + so, brsrc);
    }
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int r16 = lane & 15, kg = lane >> 4;
  int aq[RM];   // halo quad of the lane's row for tap (0,0,0), group kg: z plane wave * ZP + i / 4
#pragma unroll
  for (int i = 0; i < RM; ++i)
    aq[i] = (wave * ZP + (i >> 2)) * RZ + (2 * (i & 3) + (r16 >> 3)) * RY + (r16 & 7) * QV + kg;
  int bq[RN];
#pragma unroll
  for (int j = 0; j < RN; ++j) {
    const int col = j * 16 + r16;
    bq[j] = col * QV + (kg ^ w2_swz(col));
  }

  PROBE_T();
  issue_x(0);
  issue_w(0, 0);
  __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0): this wave's pieces have landed
  __syncthreads();
  PROBE_T();
  for (int s = 0; s < nstage; ++s) {
    const int kz = s % 3, b = s & 1;
    const bool more = s + 1 < nstage;
    if (more) issue_w(s + 1, b ^ 1);
    const T* Wb = Wl + b * WQ * EPQ;
    V8<T> af[2][RM], bf[2][RN];
    auto rd = [&](int t9, int k) {
      const int ky = t9 / 3, kx = t9 - ky * 3;
      const int hoff = kz * RZ + ky * RY + kx * QV;
#pragma unroll
      for (int j = 0; j < RN; ++j) bf[k][j].load(Wb + (t9 * BN * QV + bq[j]) * EPQ);
#pragma unroll
      for (int i = 0; i < RM; ++i) af[k][i].load(Xl + (aq[i] + hoff) * EPQ);
    };
    rd(0, 0);
#pragma unroll
    for (int t9 = 0; t9 < 9; ++t9) {
      if (t9 < 8) rd(t9 + 1, (t9 + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j) mfma_step<T>(acc[i][j], af[t9 & 1][i], bf[t9 & 1][j]);
    }
    if (more) {
      if ((s + 1) % 3 == 0) {           // next chunk: every wave is done with this halo, then refill it
        __syncthreads();
        issue_x((s + 1) / 3);
      }
      PROBE_T();
      __builtin_amdgcn_s_waitcnt(0x0f70);
      __syncthreads();
    }
    PROBE_T();
  }

  // epilogue: acc (+bias) -> LDS tile [512 ZP voxels][BN + 8] -> 16-B stores
  __syncthreads();
  T* El = reinterpret_cast<T*>(lds4);
  constexpr int EP = BN + 8;
  static_assert(512 * ZP * EP * 2 <= (XQP + 2 * WQ) * 16, "epilogue tile must fit");
#pragma unroll
  for (int j = 0; j < RN; ++j) {
    const int col = j * 16 + r16;
    const float bv = (g.bias && n0 + col < g.Ncols) ? g.bias[n0 + col] : 0.f;
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        El[((wave * ZP + (i >> 2)) * 64 + 16 * (i & 3) + 4 * kg + r) * EP + col] = from_f<T>(acc[i][j][r] + bv);
  }
  __syncthreads();
  constexpr int CG = BN / 8;
#pragma unroll
  for (int k = 0; k < ZP * CG; ++k) {
    const int e = tid + k * 512;
    const int v = e / CG, cg = e % CG;
    const int z = z0 + (v >> 6), y = y0 + ((v >> 3) & 7), x = x0 + (v & 7);
    V8<T> o;
    o.load(El + v * EP + cg * 8);
    o.store(out_at<T>(g, nbase + z * HW + (long long)y * g.W + x, n0 + cg * 8));
  }
  PROBE_T();
  PROBE_BLOCK(true);
}
// PIPE: the fragment reads of the next (dy plane, tap) step are issued before the current step's MFMAs
// MTC < MT: only the first MTC 16-row tiles are multiplied (the rest are output-channel padding, WgradArgs::pad16);
// staging and the epilogue keep the MT-row layout, the skipped rows' accumulators stay zero
template <int MT, bool NORM = false, int NST = 3, bool PIPE = false, int MTC = MT>
__global__ __launch_bounds__(512, 1) void wgrad_dma_kernel(WgradArgs g) {
  typedef bf16_t T;
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  constexpr int CO = MT * 16;
  constexpr int DCH = CO / 8, XCH = CK / 8;             // 16-B chunks per dy / halo row
  constexpr int NDI = 128 * DCH / 64;                   // dy wave-instructions per brick (8 / 16)
  constexpr int NXI = (HLO_V * XCH + 63) / 64;          // halo wave-instructions (23, the last one half)
  constexpr int NI = NDI + NXI, KI = (NI + 7) / 8;      // per brick; per wave (8 waves)
  constexpr int DS = 128 * CO, XS = NXI * 64 * 8;       // elements per stage (halo padded to whole instructions)
  constexpr int SS = DS + XS;
  __shared__ __attribute__((aligned(16))) T st[NST * SS];   // ring of NST stage images

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cin = 8 << g.cpg_shift;
  const int nchunk = wgrad_nchunk(g.cpg_shift, g.kchunks), rt_n = g.Ca / CO;
  const int tile = g.swz ? xcd_swizzle(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int ct = tile % nchunk, rt = (tile / nchunk) % rt_n, ks = tile / (nchunk * rt_n);
  const int bz_n = g.D / BRK_Z, by_n = g.H / BRK_Y, bx_n = g.W / BRK_X;
  const int nbrick = (int)(g.V / ((long long)g.D * g.H * g.W)) * bz_n * by_n * bx_n;
  const int bpk = (nbrick + g.ksplit - 1) / g.ksplit;
  const int b_begin = ks * bpk;
  const int b_end = b_begin + bpk < nbrick ? b_begin + bpk : nbrick;
  const int HW = g.H * g.W;
  const int row0 = rt * CO, c0 = ct * CK;
  const bool do_bias = g.bias_part != nullptr && ct == 0;
  const int t_begin = wave < 3 ? 4 * wave : 12 + 3 * (wave - 3);
  const int t_cnt = wave < 3 ? 4 : 3;
  const bool bias_wave = do_bias && wave == 7;

  const wd_rsrc_t drsrc = wd_rsrc(g.a, (uint32_t)(g.V * g.lda * 2));
  const wd_rsrc_t xrsrc = wd_rsrc(g.b, (uint32_t)(g.V * g.ldb * 2));

  // per DMA slot k (wave-instruction m = wave + 8 k): the lane's byte offset from the brick origin and, for a
  // halo chunk, its halo position (hz, hy, hx packed; 0xff: no chunk)
  uint32_t rel[KI], hpos[KI];
  int nw = 0;
#pragma unroll
  for (int k = 0; k < KI; ++k) {
    const int m = wave + 8 * k;
    rel[k] = 0;
    hpos[k] = 0xffu;
    if (m < NDI) {
      const int p = m * 64 + lane, v = p / DCH, c = p % DCH;
      const int gi = (c >> 1) ^ (DCH == 4 ? (v >> 2) & 1 : (v >> 1) & 3), cc = (gi << 1) | (c & 1);
      rel[k] = (uint32_t)((((v >> 5) * HW + ((v >> 3) & 3) * g.W + (v & 7)) * g.lda + row0 + cc * 8) * 2);
      ++nw;
    } else if (m < NI) {
      const int p = (m - NDI) * 64 + lane, h = p >> 2, c = p & 3;
      if (h < HLO_V) {
        const int hx = h % HLO_X, hy = (h / HLO_X) % HLO_Y, hz = h / (HLO_X * HLO_Y);
        const int cc = (((c >> 1) ^ ((hx >> 2) & 1)) << 1) | (c & 1);
        rel[k] = (uint32_t)(((hz * HW + hy * g.W + hx) * g.ldb + c0 + cc * 8) * 2);
        hpos[k] = (uint32_t)(hz | (hy << 8) | (hx << 16));
      }
      ++nw;
    }
  }
  // brick b's origin: x fastest
  auto brick_at = [&](int b, int& n, int& z0, int& y0, int& x0) __attribute__((always_inline)) {
    int q = b;
    const int bx = q % bx_n;
    q /= bx_n;
    const int by = q % by_n;
    q /= by_n;
    const int bz = q % bz_n;
    n = q / bz_n;
    z0 = bz * BRK_Z, y0 = by * BRK_Y, x0 = bx * BRK_X;
  };
  auto issue = [&](T* dst, int b) __attribute__((always_inline)) {
    int n, z0, y0, x0;
    brick_at(b, n, z0, y0, x0);
    const int vb = (n * g.D + z0) * HW + y0 * g.W + x0;
    const int dbase = vb * g.lda * 2;
    const int xbase = (vb - HW - g.W - 1) * g.ldb * 2;
#pragma unroll
    for (int k = 0; k < KI; ++k) {
      const int m = wave + 8 * k;
      if (m < NDI) {
        wd_dma16(__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)(lds_ptr_t)(dst + m * 512)),
                 (uint32_t)(dbase + (int)rel[k]), drsrc);
      } else if (m < NI) {
        const uint32_t hp = hpos[k];
        const int z = z0 - 1 + (int)(hp & 0xff), y = y0 - 1 + (int)((hp >> 8) & 0xff), x = x0 - 1 + (int)(hp >> 16);
        const bool ok = hp != 0xffu && (unsigned)z < (unsigned)g.D && (unsigned)y < (unsigned)g.H &&
                        (unsigned)x < (unsigned)g.W;
        wd_dma16(__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)(lds_ptr_t)(dst + DS + (m - NDI) * 512)),
                 ok ? (uint32_t)(xbase + (int)rel[k]) : WD_OOB, xrsrc);
      }
    }
  };
  // this wave's DMAs of all but the last brick issued have landed (vmcnt <= nw)
  // wait until at most `later` bricks' DMAs of this wave are in flight (vmcnt <= later * nw)
  auto wait_bricks = [&](int later) __attribute__((always_inline)) {
    switch (later * nw) {
#define MMSEG_WD_WAIT(N) \
  case N: __builtin_amdgcn_s_waitcnt(0x0f70 | N); break;
      MMSEG_WD_WAIT(1) MMSEG_WD_WAIT(2) MMSEG_WD_WAIT(3) MMSEG_WD_WAIT(4) MMSEG_WD_WAIT(5) MMSEG_WD_WAIT(6)
      MMSEG_WD_WAIT(7) MMSEG_WD_WAIT(8) MMSEG_WD_WAIT(9) MMSEG_WD_WAIT(10) MMSEG_WD_WAIT(11) MMSEG_WD_WAIT(12)
      MMSEG_WD_WAIT(13) MMSEG_WD_WAIT(14) MMSEG_WD_WAIT(15)
#undef MMSEG_WD_WAIT
      default: __builtin_amdgcn_s_waitcnt(0x0f70); break;
    }
  };
  // NORM: thread owns channel group cg = tid & 3 of halo rows (tid >> 2) + 128 k
  int norm_n = -1;
  float nmu[NORM ? 8 : 1], nrs[NORM ? 8 : 1];
  auto normalize = [&](T* dst, int b) __attribute__((always_inline)) {
    if constexpr (NORM) {
      int q = b;
      const int bx = q % bx_n;
      q /= bx_n;
      const int by = q % by_n;
      q /= by_n;
      const int bz = q % bz_n;
      const int n = q / bz_n;
      if (n != norm_n) {
        norm_n = n;
        const int cb = n * cin + c0 + (tid & 3) * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          nmu[j] = g.nmean[cb + j];
          nrs[j] = g.nrstd[cb + j];
        }
      }
      const int z0 = bz * BRK_Z, y0 = by * BRK_Y, x0 = bx * BRK_X, cg = tid & 3;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int h = (tid >> 2) + 128 * k;
        if (h < HLO_V) {
          const int hx = h % HLO_X, hy = (h / HLO_X) % HLO_Y, hz = h / (HLO_X * HLO_Y);
          if ((unsigned)(z0 - 1 + hz) < (unsigned)g.D && (unsigned)(y0 - 1 + hy) < (unsigned)g.H &&
              (unsigned)(x0 - 1 + hx) < (unsigned)g.W) {
            const int c = (((cg >> 1) ^ ((hx >> 2) & 1)) << 1) | (cg & 1);
            T* p = dst + DS + h * CK + c * 8;
            V8<T> v;
            v.load(p);
            norm_relu8<T>(v, nmu, nrs);
            v.store(p);
          }
        }
      }
    }
  };

  f32x4 acc[4][MT][2];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[t][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // fragment addressing (bytes): dy rows v_lo = kk + 16 (g4 >> 1) + 4 (g4 & 1) + q and v_lo + 8 share the
  // swizzle; halo rows hlo + tap offset share hx's
  const int g4 = lane >> 4, i16 = lane & 15, q4 = i16 >> 2, p4 = i16 & 3;
  const int v0 = 16 * (g4 >> 1) + 4 * (g4 & 1) + q4;
  const int dsw = DCH == 4 ? (v0 >> 2) & 1 : (v0 >> 1) & 3;
  const int hx0 = 4 * (g4 & 1) + q4;   // x of v_lo; y = 2 (g4 >> 1)
  const int hlo0 = (2 * (g4 >> 1)) * HLO_X + hx0;
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (__bf16)1.0f;
  // halo row of tap (kz, ky, kx) for the lane's voxels in brick z-plane vz
  auto xrow = [&](const char* Xb, int sb, int vz, int kz, int ky, int kx) __attribute__((always_inline)) {
    (void)sb;
    return Xb + (hlo0 + (vz + kz) * (HLO_Y * HLO_X) + ky * HLO_X + kx) * (CK * 2);
  };
  auto compute = [&](const T* S, int sb) __attribute__((always_inline)) {
    const char* Db = reinterpret_cast<const char*>(S);
    const char* Xb = reinterpret_cast<const char*>(S + DS);
#pragma unroll
    for (int kk = 0; kk < 128; kk += 32) {
      bf16x8 af[MT];
#pragma unroll
      for (int i = 0; i < MTC; ++i) {
        const bf16_t* base = reinterpret_cast<const bf16_t*>(Db + (kk + v0) * (CO * 2) + 32 * (i ^ dsw) + 8 * p4);
        af[i] = tr_frag(base, base + 8 * CO);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (t < t_cnt) {
          const int tap = t_begin + t;
          const int kz = tap / 9, ky = (tap / 3) % 3, kx = tap % 3;
          const char* row = xrow(Xb, sb, kk >> 5, kz, ky, kx);
          const int xs = ((hx0 + kx) >> 2) & 1;
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const bf16_t* pl = reinterpret_cast<const bf16_t*>(row + 32 * (j ^ xs) + 8 * p4);
            const bf16x8 bfr = tr_frag(pl, pl + HLO_X * CK);
#pragma unroll
            for (int i = 0; i < MTC; ++i)
              acc[t][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr, acc[t][i][j], 0, 0, 0);
          }
        } else if (t == 3 && bias_wave) {
#pragma unroll
          for (int i = 0; i < MTC; ++i)
            acc[3][i][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], ones, acc[3][i][0], 0, 0, 0);
        }
      }
    }
  };
  // software-pipelined: steps s = (kk, t) over this wave's TC taps, fragments double-buffered
  auto compute_pipe = [&](const T* S, int sb, auto tcc) __attribute__((always_inline)) {
    constexpr int TC = decltype(tcc)::value;
    const char* Db = reinterpret_cast<const char*>(S);
    const char* Xb = reinterpret_cast<const char*>(S + DS);
    constexpr int PD = 3;
    bf16x8 af[2][MT], bf[PD][2];
    auto load_a = [&](int kk, bf16x8(&a)[MT]) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < MTC; ++i) {
        const bf16_t* base = reinterpret_cast<const bf16_t*>(Db + (kk + v0) * (CO * 2) + 32 * (i ^ dsw) + 8 * p4);
        a[i] = tr_frag(base, base + 8 * CO);
      }
    };
    auto load_b = [&](int kk, int t, bf16x8(&b)[2]) __attribute__((always_inline)) {
      const int tap = t_begin + t;
      const int kz = tap / 9, ky = (tap / 3) % 3, kx = tap % 3;
      const char* row = xrow(Xb, sb, kk >> 5, kz, ky, kx);
      const int xs = ((hx0 + kx) >> 2) & 1;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const bf16_t* pl = reinterpret_cast<const bf16_t*>(row + 32 * (j ^ xs) + 8 * p4);
        b[j] = tr_frag(pl, pl + HLO_X * CK);
      }
    };
    // B fragments PD - 1 steps ahead (ring of PD), A one dy plane ahead
    constexpr int NS = 4 * TC;
    load_a(0, af[0]);
#pragma unroll
    for (int s0 = 0; s0 < PD - 1; ++s0)
      if (s0 < NS) load_b(32 * (s0 / TC), s0 % TC, bf[s0 % PD]);
#pragma unroll
    for (int sidx = 0; sidx < NS; ++sidx) {
      const int k4 = sidx / TC, t = sidx % TC;
      const int sn = sidx + PD - 1;
      if (sn < NS) load_b(32 * (sn / TC), sn % TC, bf[sn % PD]);
      if (t == 0 && k4 + 1 < 4) load_a(32 * (k4 + 1), af[(k4 + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < MTC; ++i)
          acc[t][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[k4 & 1][i], bf[sidx % PD][j], acc[t][i][j], 0, 0,
                                                                 0);
      if (TC == 3 && t == 2 && bias_wave) {
#pragma unroll
        for (int i = 0; i < MTC; ++i)
          acc[3][i][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[k4 & 1][i], ones, acc[3][i][0], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // prologue: bricks b_begin .. b_begin + NST - 2 in flight, the first one landed
  for (int k = 0; k < NST - 1; ++k) {
    if (b_begin + k < b_end) issue(st + k * SS, b_begin + k);
  }
  {
    const int inflight = b_end - b_begin - 1 < NST - 2 ? b_end - b_begin - 1 : NST - 2;
    wait_bricks(inflight > 0 ? inflight : 0);
  }
  __syncthreads();
  if constexpr (NORM) {
    if (b_begin < b_end) {
      normalize(st, b_begin);
      __syncthreads();
    }
  }
  // PIPE: the brick loop is instantiated per tap count (a branch on t_cnt inside it merges the two multiplies'
  // accumulator registers at every brick: copies around every MFMA group)
  auto brick_loop = [&](auto tcc) __attribute__((always_inline)) {
  for (int b = b_begin, sc = 0; b < b_end; ++b, sc = sc + 1 == NST ? 0 : sc + 1) {
    // issue brick b + NST - 1 into the stage brick b - 1 used (every wave passed the barrier after it)
    const int sn = sc == 0 ? NST - 1 : sc - 1;
    if (b + NST - 1 < b_end && g.dbg != 1) issue(st + sn * SS, b + NST - 1);
    const int sb = 0;
    if (g.dbg != 2) {
      if constexpr (PIPE)
        compute_pipe(st + sc * SS, sb, tcc);
      else
        compute(st + sc * SS, sb);
    }
    // brick b + 1 has landed once at most min(NST - 2, bricks issued after it) bricks are in flight
    {
      const int after = b_end - b - 2 < NST - 2 ? b_end - b - 2 : NST - 2;
      wait_bricks(after > 0 ? after : 0);
    }
    __syncthreads();
    if constexpr (NORM) {
      if (b + 1 < b_end) {
        normalize(st + (sc + 1 == NST ? 0 : sc + 1) * SS, b + 1);
        __syncthreads();
      }
    }
  }
  };
  if (!PIPE || t_cnt == 4)
    brick_loop(std::integral_constant<int, 4>{});
  else
    brick_loop(std::integral_constant<int, 3>{});

  static_assert(sizeof(st) >= 16 * WEP_P * sizeof(float),
                "epilogue staging must fit the stage ring");
  if (g.frag && !(g.grad != nullptr && g.ksplit == 1)) {
    // split partials in the accumulators' own layout: every (tap, i, j) fragment is 1 KB contiguous (lane l's
    // f32x4 at 16 l), so each wave stores straight from registers with 16-B lanes -- no LDS transpose, no
    // barriers; wgrad_reduce_kernel (frag_mt) maps the layout to the torch order and sums in the same fixed
    // split order as before (bitwise the same gradient)
    float* base = g.part + (long long)ks * g.Ca * g.Ncols + (long long)(rt * nchunk + ct) * (CO * 27 * CK);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (t >= t_cnt) continue;
      const int tap = t_begin + t;
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          *reinterpret_cast<f32x4*>(base + ((tap * MT + i) * 2 + j) * 256 + lane * 4) = acc[t][i][j];
    }
  } else {
    __syncthreads();
    wgrad_store_chmajor<MT>(acc, t_begin, t_cnt, reinterpret_cast<float*>(st),
                            g, ks, row0, c0);
  }
  if (bias_wave && i16 == 0) {
    // acc[3][i][0][r] = sum over the block's voxels of dy[.][row0 + 16 i + 4 g4 + r] (every column alike)
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = row0 + 16 * i + 4 * g4 + r;
        const float s = acc[3][i][0][r];
        if (g.bias_grad != nullptr && g.ksplit == 1)
          g.bias_grad[co] = g.accumulate ? g.bias_grad[co] + s : s;
        else
          g.bias_part[(long long)ks * g.Ca + co] = s;
      }
  }
}

// ------------------------------------------- row-slab weight gradient (3^3, bf16, 32 co, W % 32 == 0)
// The 96^3 32-output-channel layers' weight gradient as long-lived blocks that walk columns of x rows.
// GEMM view: dW[co][ci][tap] = sum_v dy[v][co] x[v + tap][ci].  One MFMA K-slab is 32 CONSECUTIVE x voxels of one
// (z, y) row.  The B fragment of tap (kz, ky, kx) for the dy row at (z, y) is then the halo row at (z + kz - 1,
// y + ky - 1) shifted by kx: the same fragment serves every (dy row, kz, ky) pair that lands on the same halo row.
// A wave owns one kx, one 16-channel ci half and one 16-channel co half (12 waves) and ALL nine (kz, ky) of it, so
// each halo-row fragment it reads from LDS feeds up to nine MFMAs and each dy fragment (kept in registers while
// its plane is in the 3-plane tap window) up to nine: ~0.28 LDS fragments per MFMA against 0.65 for the brick
// kernels (wgrad_brick2 / wgrad_dma: each halo fragment feeds 2 MFMAs, DESIGN (d) 8a).
// A block owns a contiguous range of dy-plane steps: columns (sample n, RY = 6 y rows (4 where H % 6 != 0), 32 x)
// walked along z, so a halo plane is staged ONCE per column (8 rows x 34 voxels for 6 x 32 dy voxels: 1.4x the x
// bytes, against 2.8x for a 4 x 4 x 8 brick's halo).  Step u of a column segment stages halo plane z_a - 1 + u and dy plane z_a + u
// into one slot of a 4-slot LDS ring by LDS-DMA (buffer_load ... lds; the same 32-B XOR swizzle as wgrad_dma,
// conflict-free for every kx shift) three steps ahead; the multiply pairs the halo plane with the dy planes
// u, u - 1, u - 2 (kz = 0, 1, 2), whose fragments rotate through three register sets.  One barrier per step.
// NORM (deferred InstanceNorm + ReLU of x): each wave normalises, in place, the halo chunks its OWN DMA
// instructions brought in (its own vmcnt orders them), one step before they are multiplied: no extra barrier.
// Bias gradient: dy fragments times a ones fragment, dealt round-robin over the six waves of a co half.
// Partials: the fragment-native layout of wgrad_dma (WReduceArgs::frag_mt = 2), summed by the same reduce.
constexpr int WROW_HX = 34;                                  // voxels per halo row
constexpr int WROW_WAVES = 12;                               // (kx, ci half, co half)
constexpr int WROW_MAXN = 16;                                // samples whose norm statistics fit the LDS table
// per plane step of RY dy rows: halo rows, halo / dy DMA wave-instructions, slot geometry (bytes)
template <int RY>
struct WRowGeo {
  static constexpr int HY = RY + 2;
  static constexpr int HI = (HY * WROW_HX * 4 + 63) / 64;   // halo chunks (16 B) / 64 lanes (RY 4: 13)
  static constexpr int DI = RY * 32 * 4 / 64;                // dy (RY 4: 8)
  static constexpr int NI = HI + DI;
  static constexpr int KI = (NI + WROW_WAVES - 1) / WROW_WAVES;   // DMA instructions per wave per step (at most)
  static constexpr int DOFF = HI * 1024;                     // dy image offset in a slot
  static constexpr int SLOT = NI * 1024;
};

// a column segment of a block's step range: column col (sample, 4 y rows, 32 x), dy planes [za, za + L)
struct WRowSeg {
  int s, col, za, L;
};

// RY dy rows per step (4 or 6; 8 spills at 168 VGPRs), NST ring slots (DMA NST - 1 steps ahead)
template <bool NORM, int RY = 6, int NST = 4>
__global__ __launch_bounds__(768, 1) void wgrad_row_kernel(WgradArgs g) {
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  typedef WRowGeo<RY> G;
  constexpr int WROW_RY = RY, WROW_HY = G::HY, WROW_HI = G::HI, WROW_NI = G::NI, WROW_DOFF = G::DOFF;
  constexpr int WROW_SLOT = G::SLOT, WROW_NST = NST, KI = G::KI;
  __shared__ __attribute__((aligned(16))) char ring[WROW_NST * WROW_SLOT];
  __shared__ __attribute__((aligned(16))) float ntab[NORM ? 2 * WROW_MAXN * CK : 4];
  __shared__ float bred[WROW_WAVES * 16];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kx = wave >> 2, jh = (wave >> 1) & 1, ih = wave & 1;   // the wave's tap column, ci half, co half
  const int cin = 8 << g.cpg_shift;
  const int nchunk = wgrad_nchunk(g.cpg_shift, g.kchunks);
  const int tile = g.swz ? xcd_swizzle(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int ct = tile % nchunk, ks = tile / nchunk;
  const int c0 = ct * CK;
  const int D = g.D, H = g.H, W = g.W;
  const int ncx = W / 32, ncol = (H / WROW_RY) * ncx;
  const int N = (int)(g.V / ((long long)D * H * W));
  const int s_tot = N * ncol * D;
  const int spb = (s_tot + g.ksplit - 1) / g.ksplit;
  const int s_begin = min(ks * spb, s_tot), s_end = min(s_begin + spb, s_tot);
  const bool do_bias = g.bias_part != nullptr && ct == 0;
  const wd_rsrc_t drsrc = wd_rsrc(g.a, (uint32_t)(g.V * g.lda * 2));
  const wd_rsrc_t xrsrc = wd_rsrc(g.b, (uint32_t)(g.V * g.ldb * 2));

  // segments and halo steps: a segment of L dy planes takes L + 2 halo steps
  auto seg_at = [&](int s) __attribute__((always_inline)) {
    WRowSeg q;
    q.s = s;
    q.col = s / D;
    q.za = s - q.col * D;
    q.L = min(D, s_end - q.col * D) - q.za;
    return q;
  };
  int h_tot = 0;
  for (int s = s_begin; s < s_end;) {
    const WRowSeg q = seg_at(s);
    h_tot += q.L + 2;
    s += q.L;
  }

  // the wave's DMA instructions (m = wave, wave + 12 < WROW_NI): m < WROW_HI halo chunks, else dy chunks.  Per
  // instruction: the lane's byte offset from the plane origin and its (y, x) position in the plane
  int nw = 0;
  int rel[KI], py[KI], px[KI], ncc[KI];
#pragma unroll
  for (int k = 0; k < KI; ++k) {
    const int m = wave + 12 * k;
    rel[k] = 0, py[k] = 0xff, px[k] = 0, ncc[k] = 0;
    if (m < WROW_HI) {
      const int p = m * 64 + lane, hy = p / (WROW_HX * 4), r = p - hy * (WROW_HX * 4), xh = r >> 2, cs = r & 3;
      const int cc = (((cs >> 1) ^ ((xh >> 2) & 1)) << 1) | (cs & 1);
      if (hy < WROW_HY) {
        rel[k] = ((hy * W + xh) * g.ldb + c0 + cc * 8) * 2;
        py[k] = hy, px[k] = xh, ncc[k] = cc;
      }
    } else if (m < WROW_NI) {
      const int p = (m - WROW_HI) * 64 + lane, ry = p >> 7, r = p & 127, x = r >> 2, cs = r & 3;
      const int cc = (((cs >> 1) ^ ((x >> 2) & 1)) << 1) | (cs & 1);
      rel[k] = ((ry * W + x) * g.lda + cc * 8) * 2;
    }
    if (m < WROW_NI) ++nw;
  }
  // DMA of halo step (segment q, step u) into ring slot `slot`
  auto issue = [&](int slot, const WRowSeg& q, int u) __attribute__((always_inline)) {
    const int n = q.col / ncol, cr = q.col - n * ncol, by = cr / ncx;
    const int y0 = by * WROW_RY, x0 = (cr - by * ncx) * 32;
    const int zh = q.za - 1 + u, zd = q.za + u;
    const bool zh_ok = (unsigned)zh < (unsigned)D, zd_ok = u < q.L;
    const int hb = (((n * D + zh) * H + (y0 - 1)) * W + (x0 - 1)) * g.ldb * 2;
    const int db = (((n * D + zd) * H + y0) * W + x0) * g.lda * 2;
    const uint32_t lbase = (uint32_t)(uintptr_t)(lds_ptr_t)(ring + slot * WROW_SLOT);
#pragma unroll
    for (int k = 0; k < KI; ++k) {
      const int m = wave + 12 * k;
      if (m < WROW_HI) {
        const int y = y0 - 1 + py[k], x = x0 - 1 + px[k];
        const bool ok = zh_ok && py[k] != 0xff && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
        wd_dma16(__builtin_amdgcn_readfirstlane(lbase + m * 1024), ok ? (uint32_t)(hb + rel[k]) : WD_OOB, xrsrc);
      } else if (m < WROW_NI) {
        wd_dma16(__builtin_amdgcn_readfirstlane(lbase + m * 1024), zd_ok ? (uint32_t)(db + rel[k]) : WD_OOB, drsrc);
      }
    }
  };
  auto wait_cnt = [&](int cnt) __attribute__((always_inline)) {
    switch (cnt) {
#define MMSEG_WR_WAIT(N) \
  case N: __builtin_amdgcn_s_waitcnt(0x0f70 | N); break;
      MMSEG_WR_WAIT(1) MMSEG_WR_WAIT(2) MMSEG_WR_WAIT(3) MMSEG_WR_WAIT(4) MMSEG_WR_WAIT(5) MMSEG_WR_WAIT(6)
      MMSEG_WR_WAIT(7) MMSEG_WR_WAIT(8) MMSEG_WR_WAIT(9) MMSEG_WR_WAIT(10) MMSEG_WR_WAIT(11) MMSEG_WR_WAIT(12)
      MMSEG_WR_WAIT(13) MMSEG_WR_WAIT(14) MMSEG_WR_WAIT(15)
#undef MMSEG_WR_WAIT
      default: __builtin_amdgcn_s_waitcnt(0x0f70); break;
    }
  };
  // NORM: relu((x - mean) * rstd) of the in-volume halo chunks this wave's own DMA brought into `slot`
  auto normalize = [&](int slot, const WRowSeg& q, int u) __attribute__((always_inline)) {
    if constexpr (NORM) {
      const int n = q.col / ncol, cr = q.col - n * ncol, by = cr / ncx;
      const int y0 = by * WROW_RY, x0 = (cr - by * ncx) * 32;
      const int zh = q.za - 1 + u;
      if ((unsigned)zh >= (unsigned)D) return;
#pragma unroll
      for (int k = 0; k < KI; ++k) {
        const int m = wave + 12 * k;
        if (m < WROW_HI) {
          const int y = y0 - 1 + py[k], x = x0 - 1 + px[k];
          if (py[k] != 0xff && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W) {
            bf16_t* p = reinterpret_cast<bf16_t*>(ring + slot * WROW_SLOT + m * 1024 + lane * 16);
            const float4* mu4 = reinterpret_cast<const float4*>(ntab + n * CK + ncc[k] * 8);
            const float4* rs4 = reinterpret_cast<const float4*>(ntab + WROW_MAXN * CK + n * CK + ncc[k] * 8);
            const float4 ma = mu4[0], mb = mu4[1], ra = rs4[0], rb = rs4[1];
            const float mu[8] = {ma.x, ma.y, ma.z, ma.w, mb.x, mb.y, mb.z, mb.w};
            const float rs[8] = {ra.x, ra.y, ra.z, ra.w, rb.x, rb.y, rb.z, rb.w};
            V8<bf16_t> v;
            v.load(p);
            norm_relu8<bf16_t>(v, mu, rs);
            v.store(p);
          }
        }
      }
    }
  };

  // fragments: lane rows x = v0 and v0 + 8 of a 32-voxel row (wgrad_dma's lane order), granule swizzle (x >> 2) & 1
  const int g4 = lane >> 4, i16 = lane & 15, q4 = i16 >> 2, p4 = i16 & 3;
  const int v0 = 16 * (g4 >> 1) + 4 * (g4 & 1) + q4;
  const int aoff = WROW_DOFF + v0 * 64 + 32 * (ih ^ (g4 & 1)) + 8 * p4;                      // + ry * 2048
  const int boff = (v0 + kx) * 64 + 32 * (jh ^ (((v0 + kx) >> 2) & 1)) + 8 * p4;            // + hy * 2176
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (__bf16)1.0f;
  f32x4 acc[3][3], accb = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};
  bf16x8 areg[3][WROW_RY];   // dy fragments of the three dy planes in the tap window (register set = plane % 3)
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int r = 0; r < WROW_RY; ++r) areg[a][r] = ones;

  if (s_begin < s_end) {
    if constexpr (NORM) {
      for (int e = tid; e < N * CK; e += 768) {
        const int n = e / CK, c = e - n * CK;
        ntab[n * CK + c] = g.nmean[n * cin + c0 + c];
        ntab[WROW_MAXN * CK + n * CK + c] = g.nrstd[n * cin + c0 + c];
      }
      __syncthreads();
    }
    // prologue: halo steps 0 .. NST - 2 issued; the DMA cursor (dq, du) points at the next step to issue
    WRowSeg dq = seg_at(s_begin);
    int du = 0;
    auto dma_next = [&]() __attribute__((always_inline)) {
      if (++du == dq.L + 2) {
        du = 0;
        if (dq.s + dq.L < s_end) dq = seg_at(dq.s + dq.L);
      }
    };
    int h_iss = 0;
    for (; h_iss < WROW_NST - 1 && h_iss < h_tot; ++h_iss) {
      issue(h_iss % WROW_NST, dq, du);
      dma_next();
    }
    wait_cnt(nw * (min(h_tot - 1, WROW_NST - 2)));
    normalize(0, seg_at(s_begin), 0);
    __syncthreads();

    int h = 0;
    // one halo step: issue step h + NST - 1, multiply step h, normalise step h + 1, barrier
    auto step = [&](auto phc, const WRowSeg& q, int u) __attribute__((always_inline)) {
      constexpr int PH = decltype(phc)::value;
      if (h_iss < h_tot) {
        issue(h_iss % WROW_NST, dq, du);
        dma_next();
        ++h_iss;
      }
      const char* S = ring + (h % WROW_NST) * WROW_SLOT;
      bf16x8 bfr[WROW_HY];
#pragma unroll
      for (int hy = 0; hy < WROW_HY; ++hy) {
        const bf16_t* pl = reinterpret_cast<const bf16_t*>(S + hy * (WROW_HX * 64) + boff);
        bfr[hy] = tr_frag(pl, pl + 8 * 32);
      }
      const bool anew = u < q.L;
      if (anew) {
#pragma unroll
        for (int r = 0; r < WROW_RY; ++r) {
          const bf16_t* pa = reinterpret_cast<const bf16_t*>(S + r * (32 * 64) + aoff);
          areg[PH][r] = tr_frag(pa, pa + 8 * 32);
        }
      }
      auto mm = [&](auto kzc, const bf16x8(&a)[WROW_RY]) __attribute__((always_inline)) {
        constexpr int KZ = decltype(kzc)::value;
#pragma unroll
        for (int hy = 0; hy < WROW_HY; ++hy)
#pragma unroll
          for (int ky = 0; ky < 3; ++ky) {
            const int ry = hy - ky;
            if (ry >= 0 && ry < WROW_RY)
              acc[KZ][ky] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ry], bfr[hy], acc[KZ][ky], 0, 0, 0);
          }
      };
      // kz = 2: dy plane u - 2 (register set (PH + 1) % 3), kz = 1: plane u - 1 ((PH + 2) % 3), kz = 0: plane u
      if (u >= 2) mm(std::integral_constant<int, 2>{}, areg[(PH + 1) % 3]);
      if (u >= 1 && u <= q.L) mm(std::integral_constant<int, 1>{}, areg[(PH + 2) % 3]);
      if (anew) {
        mm(std::integral_constant<int, 0>{}, areg[PH]);
        if (do_bias && h % 6 == kx * 2 + jh) {
#pragma unroll
          for (int r = 0; r < WROW_RY; ++r) accb = __builtin_amdgcn_mfma_f32_16x16x32_bf16(areg[PH][r], ones, accb, 0, 0, 0);
        }
      }
      // step h + 1 landed (this wave's part), normalised, then visible to all after the barrier
      wait_cnt(nw * (min(h_tot - 1, h + WROW_NST - 1) - (h + 1)));
      if (h + 1 < h_tot) {
        if (u + 1 < q.L + 2)
          normalize((h + 1) % WROW_NST, q, u + 1);
        else if (q.s + q.L < s_end)
          normalize((h + 1) % WROW_NST, seg_at(q.s + q.L), 0);
      }
      __syncthreads();
      ++h;
    };
    for (int s = s_begin; s < s_end;) {
      const WRowSeg q = seg_at(s);
      for (int u0 = 0; u0 < q.L + 2; u0 += 3) {
        step(std::integral_constant<int, 0>{}, q, u0);
        if (u0 + 1 < q.L + 2) step(std::integral_constant<int, 1>{}, q, u0 + 1);
        if (u0 + 2 < q.L + 2) step(std::integral_constant<int, 2>{}, q, u0 + 2);
      }
      s += q.L;
    }
  }

  // split partials in wgrad_dma's fragment-native layout: (tap, co tile, ci tile) fragments of 1 KB
  float* base = g.part + (long long)ks * g.Ca * g.Ncols + (long long)ct * (32 * 27 * CK);
#pragma unroll
  for (int kz = 0; kz < 3; ++kz)
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int tap = kz * 9 + ky * 3 + kx;
      *reinterpret_cast<f32x4*>(base + ((tap * 2 + ih) * 2 + jh) * 256 + lane * 4) = acc[kz][ky];
    }
  if (do_bias) {
    // accb[r] on lanes i16 == 0: sum over this wave's share of the voxels of dy[.][16 ih + 4 g4 + r]
    if (i16 == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) bred[wave * 16 + 4 * g4 + r] = accb[r];
    }
    __syncthreads();
    if (tid < 32) {
      const int i = tid >> 4;
      float sacc = 0.f;
      for (int w = i; w < WROW_WAVES; w += 2) sacc += bred[w * 16 + (tid & 15)];
      g.bias_part[(long long)ks * g.Ca + tid] = sacc;
    }
  }
}

// ------------------------------------- runtime-brick wgrad (small volumes)
// wgrad_brick2_kernel for volumes whose sides are not multiples of (4, 4, 8)
// (the 12^3 and 6^3 levels): brick (bz, by, bx) chosen on the host, <= 128
// voxels (K of one brick, zero-padded to 128) and a halo of <= 384 voxels.
// The voxel -> halo-row map of a lane does not depend on the brick, so it is
// computed once (4 k-steps x 2 rows).
constexpr int WR_MAXHV = 384;

// CB* > 0: compile-time brick (3x6x6 at the 12^3 / 6^3 levels), see conv3_brickr_kernel.
template <typename T, int MT, int CBZ = 0, int CBY = 0, int CBX = 0>
__global__ __launch_bounds__(512) void wgrad_brickr_kernel(WgradArgs g, int bz_rt, int by_rt, int bx_rt) {
  const int bz = CBZ > 0 ? CBZ : bz_rt, by = CBY > 0 ? CBY : by_rt, bx = CBX > 0 ? CBX : bx_rt;
  constexpr int EP = 16 / sizeof(T);
  constexpr int CO = MT * 16, CG = CO / 8;
  constexpr int DP = CO + EP;
  constexpr int XP = CK + EP;
  constexpr int DS = 128 * DP, XS = WR_MAXHV * XP;
  __shared__ __attribute__((aligned(16))) T lds[2 * (DS + XS)];
  constexpr int D_ITEMS = 128 * CG, X_MAX = WR_MAXHV * 4;
  constexpr int D_PER = (D_ITEMS + 511) / 512, X_PER = (X_MAX + 511) / 512;

  const T* Dy = reinterpret_cast<const T*>(g.a);
  const T* X = reinterpret_cast<const T*>(g.b);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cin = 8 << g.cpg_shift;
  const int nchunk = wgrad_nchunk(g.cpg_shift, g.kchunks), rt_n = g.Ca / CO;
  const int tile = g.swz ? xcd_swizzle(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int ct = tile % nchunk, rt = (tile / nchunk) % rt_n, ks = tile / (nchunk * rt_n);
  const int HX = bx + 2, HY = by + 2, HZ = bz + 2;
  const int HV = HZ * HY * HX, rows = bz * by * bx;
  const int bz_n = g.D / bz, by_n = g.H / by, bx_n = g.W / bx;
  const long long nbrick = (g.V / ((long long)g.D * g.H * g.W)) * bz_n * by_n * bx_n;
  // grouped: group gi's bricks (contiguous, sample-major) over its own ksplit / groups splits
  const int ngrp = g.groups > 1 ? g.groups : 1;
  const int ks_g = g.ksplit / ngrp, gi = ks / ks_g, kl = ks - gi * ks_g;
  const long long nb_g = nbrick / ngrp;
  const long long bpk = (nb_g + ks_g - 1) / ks_g;
  const long long b_begin = gi * nb_g + kl * bpk;
  const long long b_end = b_begin + bpk < (gi + 1) * nb_g ? b_begin + bpk : (gi + 1) * nb_g;
  const long long HW = (long long)g.H * g.W;
  const int row0 = rt * CO, c0 = ct * CK;
  const bool do_bias = g.bias_part != nullptr && ct == 0;
  const int t_begin = wave < 3 ? 4 * wave : 12 + 3 * (wave - 3);
  const int t_cnt = wave < 3 ? 4 : 3;

  f32x4 acc[4][MT][2];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[t][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float bsum[8] = {0, 0, 0, 0, 0, 0, 0, 0};

  auto vox_halo = [&](int v) {   // brick voxel -> halo row (tap 0); padding voxels map to row 0 (dy is 0 there)
    if (v >= rows) return 0;
    const int rx = v % bx, q = v / bx;
    return ((q / by) * HY + q % by) * HX + rx;
  };

  V8<T> dr[D_PER], xr[X_PER];
  auto load = [&](long long b) {
    int q = (int)b;   // brick index < V < 2^31 (mmseg_wgrad): 32-bit division
    const int bxi = q % bx_n;
    q /= bx_n;
    const int byi = q % by_n;
    q /= by_n;
    const int bzi = q % bz_n;
    const long long nbase = (long long)(q / bz_n) * g.D * HW;
    const int z0 = bzi * bz, y0 = byi * by, x0 = bxi * bx;
#pragma unroll
    for (int k = 0; k < D_PER; ++k) {
      const int e = tid + k * 512, v = e / CG, cg = e % CG;
      if (e < D_ITEMS) {
        if (v < rows) {
          const int rx = v % bx, qq = v / bx;
          const int ry = qq % by, rz = qq / by;
          dr[k].load(Dy + (nbase + (z0 + rz) * HW + (long long)(y0 + ry) * g.W + x0 + rx) * g.lda + row0 + cg * 8);
        } else {
          dr[k].zero();
        }
      }
    }
#pragma unroll
    for (int k = 0; k < X_PER; ++k) {
      const int e = tid + k * 512;
      if (e < HV * 4) {
        const int h = e >> 2, cg = e & 3;
        const int hx = h % HX, qq = h / HX;
        const int hy = qq % HY, hz = qq / HY;
        const int z = z0 - 1 + hz, y = y0 - 1 + hy, x = x0 - 1 + hx;
        if ((unsigned)z < (unsigned)g.D && (unsigned)y < (unsigned)g.H && (unsigned)x < (unsigned)g.W)
          xr[k].load(X + (nbase + z * HW + (long long)y * g.W + x) * g.ldb + c0 + cg * 8);
        else
          xr[k].zero();
      }
    }
  };
  auto store = [&](int buf) {
    T* Dl = lds + buf * (DS + XS);
    T* Xl = Dl + DS;
#pragma unroll
    for (int k = 0; k < D_PER; ++k) {
      const int e = tid + k * 512;
      if (e < D_ITEMS) {
        dr[k].store(Dl + (e / CG) * DP + (e % CG) * 8);
        if (do_bias) {
#pragma unroll
          for (int j = 0; j < 8; ++j) bsum[j] += dr[k].get(j);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < X_PER; ++k) {
      const int e = tid + k * 512;
      if (e < HV * 4) xr[k].store(Xl + (e >> 2) * XP + (e & 3) * 8);
    }
  };

  const int g4 = lane >> 4, i16 = lane & 15, q4 = i16 >> 2, p4 = i16 & 3;
  int hlo[4], hhi[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    hlo[s] = vox_halo(s * 32 + 8 * g4 + q4);
    hhi[s] = vox_halo(s * 32 + 8 * g4 + q4 + 4);
  }
  int toff[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int tap = t_begin + (t < t_cnt ? t : 0);
    toff[t] = ((tap / 9) * HY + (tap / 3) % 3) * HX + tap % 3;
  }
  int buf = 0;
  if (b_begin < b_end) {
    load(b_begin);
    store(0);
  }
  __syncthreads();
  for (long long b = b_begin; b < b_end; ++b) {
    const bool more = b + 1 < b_end;
    if (more) load(b + 1);
    const T* Dl = lds + buf * (DS + XS);
    const T* Xl = Dl + DS;
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        if (s * 32 >= rows) break;
        bf16x8 af[MT];
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          const bf16_t* base = (const bf16_t*)Dl + (s * 32 + 8 * g4 + q4) * DP + i * 16 + 4 * p4;
          af[i] = tr_frag(base, base + 4 * DP);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          if (t < t_cnt) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const bf16_t* pl = (const bf16_t*)Xl + (hlo[s] + toff[t]) * XP + j * 16 + 4 * p4;
              const bf16_t* ph = (const bf16_t*)Xl + (hhi[s] + toff[t]) * XP + j * 16 + 4 * p4;
              const bf16x8 bfr = tr_frag(pl, ph);
#pragma unroll
              for (int i = 0; i < MT; ++i)
                acc[t][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr, acc[t][i][j], 0, 0, 0);
            }
          }
        }
      }
    } else {
      for (int kk = 0; kk < rows; kk += 4) {
        const int v = kk + g4;
        const int hv = vox_halo(v);
        float af[MT];
#pragma unroll
        for (int i = 0; i < MT; ++i) af[i] = (float)Dl[v * DP + i * 16 + i16];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          if (t < t_cnt) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const float bv = (float)Xl[(hv + toff[t]) * XP + j * 16 + i16];
#pragma unroll
              for (int i = 0; i < MT; ++i)
                acc[t][i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bv, acc[t][i][j], 0, 0, 0);
            }
          }
        }
      }
    }
    if (more) store(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }

  static_assert(sizeof(lds) >= 16 * WEP_P * sizeof(float) && sizeof(lds) >= 512 * 8 * sizeof(float),
                "epilogue staging must fit the stage buffers");
  wgrad_store_chmajor<MT>(acc, t_begin, t_cnt, reinterpret_cast<float*>(lds), g, ks, row0, c0);
  if (do_bias) wgrad_store_bias<CG>(bsum, reinterpret_cast<float*>(lds), g, ks, row0);
}

struct WBrick { int bz, by, bx; };

// Runtime brick for the small-volume wgrad: divisors of (D, H, W), <= 128 voxels,
// halo <= WR_MAXHV; the most voxels wins.  {0,0,0} = none.
WBrick plan_wgrad_brickr(int D, int H, int W) {
  WBrick best{0, 0, 0};
  int brows = 0;
  for (int bz = 1; bz <= D && bz <= 16; ++bz) {
    if (D % bz) continue;
    for (int by = 1; by <= H && by <= 16; ++by) {
      if (H % by) continue;
      for (int bx = 1; bx <= W && bx <= 16; ++bx) {
        if (W % bx) continue;
        const int rows = bz * by * bx;
        const int halo = (bz + 2) * (by + 2) * (bx + 2);
        if (rows > 128 || halo > WR_MAXHV) continue;
        // ties go to the smaller halo (12^3: 3x6x6, the compile-time kernel, over 3x3x12)
        const bool tie_better = rows == brows && halo < (best.bz + 2) * (best.by + 2) * (best.bx + 2);
        if (rows > brows || tie_better) {
          brows = rows;
          best = {bz, by, bx};
        }
      }
    }
  }
  return brows >= 32 ? best : WBrick{0, 0, 0};
}

// part[ks][row][col] -> torch-layout gradient (fixed-order sum over ks).
//   CONV3 : grad[co][ci][tap]    row=co, col = tap*Cin_pad + ci, ci < Cin_real
//   POINT : grad[co][ci]         row=co, col = ci
//   CONVT : grad[ci][co][tap]    row=ci, col = tap*Cout + co
struct WReduceArgs {
  const float* part;
  float* grad;
  const float* bias_part;
  float* bias_grad;
  int Ca, Ncols, ksplit;
  int cpad, creal;    // per-tap channel count in cols (padded) and real count
  int ntap;           // 27 (CONV3), 1 (POINT), 8 (CONVT)
  int accumulate;
  int chmajor;        // cols are channel-major (col = c*ntap + tap, brick2/brickr partials) instead of tap-major
  int frag_mt;        // > 0: wgrad_dma's fragment-native partials (MT 16-row tiles per block), see wgrad_dma_kernel
  int nchunk;         // frag_mt > 0: 32-channel chunks per tile row
  // grouped (blockIdx.y = group gi < gridDim.y): splits [gi * ksplit, (gi + 1) * ksplit) of the partials (ksplit
  // counts one group's splits), written to grad + gi * grad_gstride / bias_grad + gi * bias_gstride
  long long grad_gstride;
  int bias_gstride;
  int vec4;           // host-set (wred_vec4): channel-major sums as 16-B stores
};

// 256 threads = (256/S) float4 columns x S split slices: slice s sums splits
// k = s, s+S, ... with 16-B loads, then the S slice sums are added in slice
// order -> deterministic.  S follows ksplit (1 for a few splits, up to 64 for
// thousands), so every thread has a few independent loads in flight.  Bias
// partials ([ks][Ca], after the weight columns) are summed by the blocks past
// the weight range.
template <int U>
__device__ __forceinline__ void wred_body(WReduceArgs g, const int S, const int bx, const int gy, float4* red) {
  if (gy) {                                   // grouped: this group's splits and gradient
    const long long gi = gy;
    g.part += gi * g.ksplit * ((long long)g.Ca * g.Ncols);
    if (g.bias_part) g.bias_part += gi * g.ksplit * g.Ca;
    g.grad += gi * g.grad_gstride;
    if (g.bias_grad) g.bias_grad += gi * g.bias_gstride;
  }
  const int NC = 256 / S;                     // float4 columns per block
  const int col4 = threadIdx.x % NC, sl = threadIdx.x / NC;
  const long long total = (long long)g.Ca * g.Ncols;   // multiple of 4
  const long long e0 = ((long long)bx * NC + col4) * 4;
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (e0 < total) {
    const float4* p = reinterpret_cast<const float4*>(g.part + e0);
    const long long stride4 = total / 4;
    // U loads in flight per thread (the sum order stays k = sl, sl + S, ...)
    for (int k0 = sl; k0 < g.ksplit; k0 += U * S) {
      float4 a[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = k0 + u * S;
        if (k < g.ksplit) a[u] = p[(long long)k * stride4];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (k0 + u * S < g.ksplit) {
          v.x += a[u].x; v.y += a[u].y; v.z += a[u].z; v.w += a[u].w;
        }
      }
    }
  } else if (g.bias_part) {
    const long long r0 = e0 - total;   // bias rows r0 .. r0+3
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (r0 + q >= g.Ca) break;
      float a = 0.f;
      for (int k = sl; k < g.ksplit; k += S) a += g.bias_part[(long long)k * g.Ca + r0 + q];
      (&v.x)[q] = a;
    }
  }
  if (S > 1) {
    // slice sums: a fixed pairwise tree (S = 16..64 made the former serial sweep of one thread per column the
    // kernel's critical path)
    red[sl * NC + col4] = v;
    __syncthreads();
#pragma unroll
    for (int h = S / 2; h > 0; h >>= 1) {
      if (sl < h) {
        const float4 a = red[(sl + h) * NC + col4];
        v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
        red[sl * NC + col4] = v;
      }
      __syncthreads();
    }
    if (sl != 0) return;
  }
  // channel-major partials: the four sums are four consecutive gradient floats (col = c ntap + tap and the torch
  // offset (row creal + c) ntap + tap differ by row (Ncols - creal ntap), a multiple of 4, and the real-channel
  // boundary col = creal ntap is one too) -- one 16-B store instead of four 4-B ones
  if (g.vec4 && e0 < total && g.frag_mt == 0 && g.chmajor) {
    const long long row = e0 / g.Ncols;
    const long long col = e0 - row * g.Ncols;
    if (col >= (long long)g.creal * g.ntap) return;   // channel padding: dropped
    float4* d = reinterpret_cast<float4*>(g.grad + row * ((long long)g.creal * g.ntap) + col);
    if (g.accumulate) {
      const float4 o = *d;
      v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
    }
    *d = v;
    return;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const long long idx = e0 + q;
    const float val = (&v.x)[q];
    if (idx >= total) {
      const long long row = idx - total;
      if (!g.bias_part || row >= g.Ca) continue;
      g.bias_grad[row] = g.accumulate ? g.bias_grad[row] + val : val;
      continue;
    }
    int row, tt, c;
    if (g.frag_mt > 0) {
      // tile (rt, ct) of CO x (27 taps x 32 channels), inside it ((tap * MT + i) * 2 + j) * 256 + lane * 4 + r
      const int CO = g.frag_mt * 16, tsz = CO * 27 * 32;
      const int tile = (int)(idx / tsz), loc = (int)(idx - (long long)tile * tsz);
      const int rt = tile / g.nchunk, ct = tile - rt * g.nchunk;
      const int f = loc >> 8, e = loc & 255, lane = e >> 2, r = e & 3;
      const int j = f & 1, i = (f >> 1) % g.frag_mt;
      tt = (f >> 1) / g.frag_mt;
      row = rt * CO + 16 * i + 4 * (lane >> 4) + r;
      c = ct * 32 + 16 * j + (lane & 15);
      if (row >= g.Ca || c >= g.creal) continue;   // past the tiles (channel padding): never written, sum dropped
      const long long dst = ((long long)row * g.creal + c) * g.ntap + tt;
      if (g.accumulate) g.grad[dst] += val;
      else g.grad[dst] = val;
      continue;
    }
    row = (int)(idx / g.Ncols);
    const int col = (int)(idx - (long long)row * g.Ncols);
    if (g.chmajor) {
      c = col / g.ntap;
      tt = col - c * g.ntap;
    } else {
      tt = col / g.cpad;
      c = col - tt * g.cpad;
    }
    if (c >= g.creal || tt >= g.ntap) continue;
    const long long dst = ((long long)row * g.creal + c) * g.ntap + tt;   // torch layout [row][c_real][tap]
    if (g.accumulate) g.grad[dst] += val;
    else g.grad[dst] = val;
  }
}

template <int S, int U = 4>
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(WReduceArgs g) {
  __shared__ float4 red[256];
  wred_body<U>(g, S, blockIdx.x, blockIdx.y, red);
}

// Several layers' split reduces in one launch (mmseg_wgrad_reduce_flush): descriptor k owns blocks
// [blk0[k], blk0[k + 1]) = groups x nbx[k], each summed exactly as its own wgrad_reduce_kernel<S[k]> launch would
// (same slices, same fixed order: bitwise the same gradient).
constexpr int WRB_MAX = 30;
struct WReduceBatch {
  int n;
  int blk0[WRB_MAX + 1];
  int nbx[WRB_MAX];
  int S[WRB_MAX];
  WReduceArgs d[WRB_MAX];
};
__global__ __launch_bounds__(256) void wgrad_reduce_batch_kernel(WReduceBatch b) {
  __shared__ float4 red[256];
  const int bid = blockIdx.x;
  int k = 0;
  while (k + 1 < b.n && bid >= b.blk0[k + 1]) ++k;
  const int local = bid - b.blk0[k];
  wred_body<4>(b.d[k], b.S[k], local % b.nbx[k], local / b.nbx[k], red);
}

// Column sums (bias gradient): db[c] = sum_v dy[v][c], split over voxels.
template <typename T>
__global__ void colsum_partial_kernel(const T* __restrict__ dy, int ld, int C, long long V, long long vps,
                                      float* __restrict__ part) {
  // block: 256 threads = (256/C8) voxel lanes x C8 channel groups (C8 = C/8 <= 64)
  const int C8 = C >> 3;
  const int lanes_v = 256 / C8;
  const int tid = threadIdx.x;
  const int cg = tid % C8, vl = tid / C8;
  const long long v0 = (long long)blockIdx.x * vps;
  long long v1 = v0 + vps;
  if (v1 > V) v1 = V;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (vl < lanes_v) {
    for (long long v = v0 + vl; v < v1; v += lanes_v) {
      V8<T> x;
      x.load(dy + v * ld + cg * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += x.get(j);
    }
  }
  __shared__ float red[256 * 8];
#pragma unroll
  for (int j = 0; j < 8; ++j) red[tid * 8 + j] = s[j];
  __syncthreads();
  if (tid < C8) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int l = 0; l < lanes_v; ++l)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += red[(l * C8 + tid) * 8 + j];
#pragma unroll
    for (int j = 0; j < 8; ++j) part[(long long)blockIdx.x * C + tid * 8 + j] = acc[j];
  }
}

// one 256-thread block per channel: threads stride over the block partials (4 loads in flight), a fixed
// shuffle tree per wave, then the 4 waves in order (one wave per channel walked ~30 dependent loads per lane
// for the transposed conv's 8 x ksplit column-sum partials)
__global__ __launch_bounds__(256) void colsum_reduce_kernel(const float* __restrict__ part, int nblk, int C,
                                                            float* __restrict__ out, int accumulate) {
  const int c = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float v = 0.f;
#pragma unroll 4
  for (int b = threadIdx.x; b < nblk; b += 256) v += part[(long long)b * C + c];
  v = wave_sum(v);
  __shared__ float wred[4];
  if (lane == 0) wred[wave] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float t = ((wred[0] + wred[1]) + wred[2]) + wred[3];
    out[c] = accumulate ? out[c] + t : t;
  }
}

// ------------------------------------------------------------ weight pack
// dst[kgi][col][j] (T), KGp x Cpad x 8, from fp32 torch-layout weights.
//   0 CONV3_FWD  : W[Co][Ci][27]; kgi = tap*(Cip/8)+c8, col = co, ci = c8*8+j
//   1 CONV3_DGRAD: kgi = tap*(Co/8)+c8, col = ci, co = c8*8+j, tap' = 26-tap
//   2 POINT_FWD  : W[Co][Ci]; kgi = c8, col = co, ci = c8*8+j
//   3 POINT_DGRAD: kgi = c8, col = ci, co = c8*8+j
//   4 CONVT_FWD  : W[Ci][Co][8]; kgi = c8 (ci), col = tap*Co + co
//   5 CONVT_DGRAD: kgi = tap*(Co/8)+c8, col = ci, co = c8*8+j
//   6 / 7        : modes 1 / 5 with Cip = the padded output-channel count (rows co >= Co zero)
struct PackArgs {
  const float* w;
  void* dst;
  int Co, Ci, Cip;  // Cip: padded input channels (multiple of 8) for CONV3_FWD
  int KG, KGp, Cpad;
};

// Value of packed element (kgi, col, j) of a mode-`mode` image (0 outside the weight).
__device__ __forceinline__ float pack_value(const float* __restrict__ w, int mode, int Co, int Ci, int Cip, int kgi,
                                            int col, int j) {
  switch (mode) {
    case 0: {
      const int cpg = Cip >> 3, t = kgi / cpg, ci = (kgi % cpg) * 8 + j, co = col;
      if (co < Co && ci < Ci) return w[((long long)co * Ci + ci) * 27 + t];
    } break;
    case 1: {
      const int cpg = Co >> 3, t = kgi / cpg, co = (kgi % cpg) * 8 + j, ci = col;
      if (ci < Ci) return w[((long long)co * Ci + ci) * 27 + (26 - t)];
    } break;
    case 2: {
      const int ci = kgi * 8 + j, co = col;
      if (co < Co && ci < Ci) return w[(long long)co * Ci + ci];
    } break;
    case 3: {
      const int co = kgi * 8 + j, ci = col;
      if (ci < Ci && co < Co) return w[(long long)co * Ci + ci];
    } break;
    case 4: {
      const int ci = kgi * 8 + j;
      const int t = col / Co, co = col % Co;
      if (t < 8 && ci < Ci) return w[((long long)ci * Co + co) * 8 + t];
    } break;
    case 5: {
      const int cpg = Co >> 3, t = kgi / cpg, co = (kgi % cpg) * 8 + j, ci = col;
      if (ci < Ci) return w[((long long)ci * Co + co) * 8 + t];
    } break;
    case 6: {   // CONV3_DGRAD over Cop = Cip padded output channels (zero rows co >= Co)
      const int cpg = Cip >> 3, t = kgi / cpg, co = (kgi % cpg) * 8 + j, ci = col;
      if (ci < Ci && co < Co) return w[((long long)co * Ci + ci) * 27 + (26 - t)];
    } break;
    case 7: {   // CONVT_DGRAD over Cop = Cip padded output channels
      const int cpg = Cip >> 3, t = kgi / cpg, co = (kgi % cpg) * 8 + j, ci = col;
      if (ci < Ci && co < Co) return w[((long long)ci * Co + co) * 8 + t];
    } break;
  }
  return 0.f;
}

template <typename T>
__global__ void pack_weight_kernel(PackArgs g, int mode) {
  long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)g.KGp * g.Cpad * 8;
  if (idx >= total) return;
  const int j = (int)(idx & 7);
  const long long q = idx >> 3;
  const int col = (int)(q % g.Cpad);
  const int kgi = (int)(q / g.Cpad);
  const float v = kgi < g.KG ? pack_value(g.w, mode, g.Co, g.Ci, g.Cip, kgi, col, j) : 0.f;
  reinterpret_cast<T*>(g.dst)[idx] = from_f<T>(v);
}

// Batched 3^3 pack: one launch writes BOTH operand images of every 3^3 conv of
// a model (forward [27*Cip/8][Cpad][8] and flipped/transposed data-gradient
// [27*Co/8][Cpad_d][8]) from ONE coalesced read of the fp32 master weights.
// Block = (8 output channels, 32 input channels) of one layer: the 8 x 32 x 27
// source floats are contiguous runs per output channel, staged in LDS, then
// written as 16-B vectors (8 input channels for the forward image, 8 output
// channels for the data-gradient image).  Entries the block does not own
// (K padding, Cin padding of the stem) are zero from allocation.
struct Pack3Desc {
  const float* w;       // [Co][Ci][27]
  void* wf;             // forward image
  void* wd;             // data-gradient image or null
  int Co, Ci, Cip, Cpad, Cpad_d;
  int block_begin;      // first block of this layer in the launch
  int Cop;              // data-gradient reduction channels (pack mode 6: padded Co; 0 = Co)
  int pad1;
};

// The two operand images of one (8 co x 32 ci) tile of a 3^3 conv's weight staged in sw[co][ci][tap] (ci >= cis
// zero): forward image (tap, 8-ci group, co) and data-gradient image (tap s -> kgi = (26 - s) * Cop/8 + co0/8,
// column ci, 8 co per vector; rows co >= Co of a padded image are zero from allocation), 16-B stores.
template <typename T>
__device__ __forceinline__ void pack3_write(const float (*sw)[33][29], void* wfp, void* wdp, int Co, int Cip, int Cpad,
                                            int Cpad_d, int Cop, int co0, int ci0, int cis) {
  const int tid = threadIdx.x;
  const int cpg = Cip >> 3;
  const int ngrp = ((Cip - ci0) < 32 ? (Cip - ci0) : 32) >> 3;
  T* wf = reinterpret_cast<T*>(wfp);
  for (int e = tid; e < 27 * 4 * 8; e += 256) {
    const int co = e & 7, cg = (e >> 3) & 3, t = e >> 5;
    if (cg >= ngrp || co0 + co >= Co) continue;
    V8<T> v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v.set(j, sw[co][cg * 8 + j][t]);
    const long long kgi = (long long)t * cpg + (ci0 >> 3) + cg;
    v.store(wf + (kgi * Cpad + co0 + co) * 8);
  }
  if (wdp == nullptr) return;
  const int cpgd = (Cop > 0 ? Cop : Co) >> 3;
  T* wd = reinterpret_cast<T*>(wdp);
  for (int e = tid; e < 27 * 32; e += 256) {
    const int ci = e & 31, t = e >> 5;
    if (ci >= cis) continue;
    V8<T> v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v.set(j, sw[j][ci][t]);
    const long long kgi = (long long)(26 - t) * cpgd + (co0 >> 3);
    v.store(wd + (kgi * Cpad_d + ci0 + ci) * 8);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void pack_conv3_batched_kernel(const Pack3Desc* __restrict__ descs, int n) {
  __shared__ float sw[8][33][29];   // padded: conflict-free image reads (the [8][32][28] form was 32-way on the forward image)
  int lo = 0, hi = n - 1;
  const int b = blockIdx.x;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (descs[mid].block_begin <= b) lo = mid;
    else hi = mid - 1;
  }
  const Pack3Desc d = descs[lo];
  const int nci = (d.Ci + 31) / 32;
  const int lb = b - d.block_begin;
  const int co0 = (lb / nci) * 8, ci0 = (lb % nci) * 32;
  const int cis = d.Ci - ci0 < 32 ? d.Ci - ci0 : 32;
  const int tid = threadIdx.x;
  if (cis == 32 && co0 + 8 <= d.Co && (d.Ci & 3) == 0) {
    // full tile: each co row of the tile is 864 contiguous floats, 16-B aligned -> float4 loads
    for (int e = tid; e < 8 * 216; e += 256) {
      const int co = e / 216, r4 = (e - co * 216) * 4;
      const float4 v = *reinterpret_cast<const float4*>(d.w + ((long long)(co0 + co) * d.Ci + ci0) * 27 + r4);
      const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int r = r4 + k, ci = r / 27, t = r - ci * 27;
        sw[co][ci][t] = vv[k];
      }
    }
  } else {
    for (int e = tid; e < 8 * 32 * 27; e += 256) {
      const int co = e / (32 * 27), r = e - co * (32 * 27);
      const int ci = r / 27, t = r - ci * 27;
      sw[co][ci][t] = (ci < cis && co0 + co < d.Co) ? d.w[((long long)(co0 + co) * d.Ci + ci0) * 27 + r] : 0.f;
    }
  }
  __syncthreads();
  pack3_write<T>(sw, d.wf, d.wd, d.Co, d.Cip, d.Cpad, d.Cpad_d, d.Cop, co0, ci0, cis);
}

// Batched pack: one launch packs every layer of a model (descriptor table in device memory).
struct PackDesc {
  const float* w;
  void* dst;
  int mode, Co, Ci, Cip, KG, KGp, Cpad, pad0;
  long long begin;   // first element (of the virtual concatenation) owned by this descriptor
};

template <typename T>
__global__ void pack_weight_batched_kernel(const PackDesc* __restrict__ descs, int n, long long total) {
  for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {                    // last descriptor with begin <= idx
      const int mid = (lo + hi + 1) >> 1;
      if (descs[mid].begin <= idx) lo = mid;
      else hi = mid - 1;
    }
    const PackDesc d = descs[lo];
    const long long li = idx - d.begin;
    const int j = (int)(li & 7);
    const long long q = li >> 3;
    const int col = (int)(q % d.Cpad);
    const int kgi = (int)(q / d.Cpad);
    const float v = kgi < d.KG ? pack_value(d.w, d.mode, d.Co, d.Ci, d.Cip, kgi, col, j) : 0.f;
    reinterpret_cast<T*>(d.dst)[li] = from_f<T>(v);
  }
}

// ------------------------------------------------------------ fused AdamW + weight pack
// The captured training step's optimizer launch (mmseg_adamw_pack_dev): the AdamW update of the whole flat arena
// (adamw_one: mmseg_adamw_dev's per-element bits) with every packed weight's NEW value also written into its
// operand images -- what mmseg_pack_conv3_batched / mmseg_pack_weights_batched would write from the updated fp32
// weights at the next forward, which then skips its pack (one read of the fp32 weights and two launches less per
// step).  Blocks by descriptor kind:
//   0  3^3 conv: (8 co x 32 ci x 27 taps) tiles, pack_conv3_batched_kernel's tiles and image writes;
//   1  1x1 / token linear W[Co][Ci] (pack modes 2 / 3) or transposed conv W[Ci][Co][8] (modes 4 / 5 / 7):
//      8 source rows x up to AP_KT columns staged in LDS, written as 16-B vectors per image;
//   2  a plain range of the arena (biases, norm / LayerNorm parameters, tables): the update only.
// The host table (engine/layers.py Packer.adam_table) covers every arena element exactly once.  Entries no block
// owns (K / channel padding) stay zero from allocation, as with the batched packs.
constexpr int AP_KT = 512;      // kind-1 tile columns (a multiple of 64: whole 8-co groups of a transposed conv)
constexpr int AP_RANGE = 4096;  // kind-2 elements per block
struct AdamPackDesc {
  void* d0;            // kind 0: forward image; kind 1: the mode0 image
  void* d1;            // data-gradient image / the mode1 image (null: none)
  long long off;       // first arena element of the weight (kind 0 / 1) or of the range (kind 2)
  int kind, block_begin;
  int R, K;            // kind 1: source rows x columns; kind 2: K = the range's length
  int mode0, mode1;    // kind 1: pack modes of d0 / d1
  int Co, Ci, Cip, Cpad, Cpad_d, Cop;   // kind 0: Pack3Desc's fields; kind 1: the weight's Co, Ci, Cpad / Cpad_d
                                        // of d0 / d1, Cop of mode 7
};

// AdamW over `rows` runs of `len` arena elements (run r starts at a0 + r * stride); the new value of element
// (r, i) goes to put(r, i, value).  float4 lanes when every run is 16-B aligned.
template <typename PUT>
__device__ __forceinline__ void ap_update(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                          float* __restrict__ v, long long a0, long long stride, int rows, int len,
                                          const AdamHyper& h, PUT&& put) {
  const int tid = threadIdx.x;
  if (((a0 | stride | (long long)len) & 3) == 0) {
    const int n4 = len >> 2, tot = rows * n4;
    for (int e = tid; e < tot; e += 256) {
      const int r = e / n4, q = e - r * n4;
      const long long k = ((a0 + r * stride) >> 2) + q;
      float4 pv = reinterpret_cast<const float4*>(p)[k];
      const float4 gv = reinterpret_cast<const float4*>(g)[k];
      float4 mv = reinterpret_cast<const float4*>(m)[k];
      float4 vv = reinterpret_cast<const float4*>(v)[k];
      adamw_one(pv.x, gv.x, mv.x, vv.x, h);
      adamw_one(pv.y, gv.y, mv.y, vv.y, h);
      adamw_one(pv.z, gv.z, mv.z, vv.z, h);
      adamw_one(pv.w, gv.w, mv.w, vv.w, h);
      reinterpret_cast<float4*>(p)[k] = pv;
      reinterpret_cast<float4*>(m)[k] = mv;
      reinterpret_cast<float4*>(v)[k] = vv;
      put(r, 4 * q, pv.x);
      put(r, 4 * q + 1, pv.y);
      put(r, 4 * q + 2, pv.z);
      put(r, 4 * q + 3, pv.w);
    }
  } else {
    const int tot = rows * len;
    for (int e = tid; e < tot; e += 256) {
      const int r = e / len, i = e - r * len;
      const long long k = a0 + r * stride + i;
      float pv = p[k], mv = m[k], vv = v[k];
      adamw_one(pv, g[k], mv, vv, h);
      p[k] = pv;
      m[k] = mv;
      v[k] = vv;
      put(r, i, pv);
    }
  }
}

// one image of a kind-1 tile: s[8][AP_KT + 1] rows r0 .. r0 + 7, columns k0 .. k0 + kt (kt8: kt rounded up to 8,
// zero past kt)
template <typename T>
__device__ __forceinline__ void ap_write1(const float (*s)[AP_KT + 1], int mode, void* dstp, int cpad, int Co, int Cop,
                                          int r0, int k0, int kt, int kt8) {
  const int tid = threadIdx.x;
  T* dst = reinterpret_cast<T*>(dstp);
  if (mode == 2) {            // 1x1 forward: (ci group, co) <- 8 ci of row co
    for (int e = tid; e < kt8; e += 256) {
      const int rr = e & 7, cg = e >> 3;
      V8<T> w;
#pragma unroll
      for (int j = 0; j < 8; ++j) w.set(j, s[rr][cg * 8 + j]);
      w.store(dst + ((long long)((k0 >> 3) + cg) * cpad + r0 + rr) * 8);
    }
  } else if (mode == 3) {     // 1x1 data gradient: (co group r0 / 8, ci) <- the tile's 8 rows of column ci
    for (int c = tid; c < kt; c += 256) {
      V8<T> w;
#pragma unroll
      for (int j = 0; j < 8; ++j) w.set(j, s[j][c]);
      w.store(dst + ((long long)(r0 >> 3) * cpad + k0 + c) * 8);
    }
  } else if (mode == 4) {     // transposed forward: (ci group r0 / 8, t Co + co) <- 8 rows of column co 8 + t
    const int ncol8 = kt >> 3;
    for (int e = tid; e < kt; e += 256) {
      const int t = e / ncol8, col = e - t * ncol8;
      V8<T> w;
#pragma unroll
      for (int j = 0; j < 8; ++j) w.set(j, s[j][col * 8 + t]);
      w.store(dst + ((long long)(r0 >> 3) * cpad + t * Co + (k0 >> 3) + col) * 8);
    }
  } else {                    // 5 / 7 transposed data gradient: (t Cop/8 + co group, ci) <- 8 co of row ci, tap t
    const int cpgd = (mode == 7 ? Cop : Co) >> 3, ngrp = kt >> 6;
    for (int e = tid; e < 64 * ngrp; e += 256) {
      const int rr = e & 7, t = (e >> 3) & 7, cg = e >> 6;
      V8<T> w;
#pragma unroll
      for (int j = 0; j < 8; ++j) w.set(j, s[rr][(cg * 8 + j) * 8 + t]);
      const int co = (k0 >> 3) + cg * 8;
      w.store(dst + ((long long)(t * cpgd + (co >> 3)) * cpad + r0 + rr) * 8);
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void adamw_pack_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                         float* __restrict__ m, float* __restrict__ v,
                                                         const AdamPackDesc* __restrict__ descs, int n,
                                                         AdamHyper hv, const AdamHyper* __restrict__ hp,
                                                         const float* __restrict__ skip) {
  __shared__ float sw[8][33][29];
  AdamHyper h;
  if (!adamw_load(hv, hp, skip, h)) return;
  int lo = 0, hi = n - 1;
  const int b = blockIdx.x;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (descs[mid].block_begin <= b) lo = mid;
    else hi = mid - 1;
  }
  const AdamPackDesc d = descs[lo];
  const int lb = b - d.block_begin;
  const int tid = threadIdx.x;
  if (d.kind == 0) {
    const int nci = (d.Ci + 31) / 32;
    const int co0 = (lb / nci) * 8, ci0 = (lb % nci) * 32;
    const int cis = d.Ci - ci0 < 32 ? d.Ci - ci0 : 32;
    if (co0 >= d.Co) return;
    for (int e = tid; e < 8 * (32 - cis) * 27; e += 256) {   // the tile's channel padding reads as zero
      const int co = e / ((32 - cis) * 27), r = e - co * ((32 - cis) * 27);
      sw[co][cis + r / 27][r % 27] = 0.f;
    }
    ap_update(p, g, m, v, d.off + ((long long)co0 * d.Ci + ci0) * 27, (long long)d.Ci * 27, 8, cis * 27, h,
              [&](int r, int i, float x) __attribute__((always_inline)) {
                const int ci = i / 27;
                sw[r][ci][i - ci * 27] = x;
              });
    __syncthreads();
    pack3_write<T>(sw, d.d0, d.d1, d.Co, d.Cip, d.Cpad, d.Cpad_d, d.Cop, co0, ci0, cis);
  } else if (d.kind == 1) {
    float (*s)[AP_KT + 1] = reinterpret_cast<float (*)[AP_KT + 1]>(&sw[0][0][0]);
    const int nkt = (d.K + AP_KT - 1) / AP_KT;
    const int r0 = (lb / nkt) * 8, k0 = (lb % nkt) * AP_KT;
    const int kt = d.K - k0 < AP_KT ? d.K - k0 : AP_KT, kt8 = (kt + 7) & ~7;
    if (r0 >= d.R) return;
    for (int e = tid; e < 8 * (kt8 - kt); e += 256) s[e / (kt8 - kt)][kt + e % (kt8 - kt)] = 0.f;
    ap_update(p, g, m, v, d.off + (long long)r0 * d.K + k0, d.K, 8, kt, h,
              [&](int r, int i, float x) __attribute__((always_inline)) { s[r][i] = x; });
    __syncthreads();
    ap_write1<T>(s, d.mode0, d.d0, d.Cpad, d.Co, d.Cop, r0, k0, kt, kt8);
    if (d.d1 != nullptr) ap_write1<T>(s, d.mode1, d.d1, d.Cpad_d, d.Co, d.Cop, r0, k0, kt, kt8);
  } else {
    if (lb * AP_RANGE >= d.K) return;
    const long long a0 = d.off + (long long)lb * AP_RANGE;
    const int len = d.K - lb * AP_RANGE < AP_RANGE ? d.K - lb * AP_RANGE : AP_RANGE;
    ap_update(p, g, m, v, a0, 0, 1, len, h, [](int, int, float) __attribute__((always_inline)) {});
  }
}

// ------------------------------------------------------------ host launch
template <typename T, int MODE>
int launch_splitk_reduce(const GemmArgs& g, hipStream_t s) {
  const long long total = (long long)g.M * g.Ncols;
  const bool vec = MODE != MODE_CONVT_FWD && splitk_vec<MODE>(g);   // (the sliced reduce: not the transposed conv)
  int S = 1;
  while (S < 16 && g.ksplit / (2 * S) >= 4) S *= 2;
  if (vec && S > 1) {
    const int nb = ceil_div(total / 4, 256 / S);
    if (S == 16) MMSEG_LAUNCH((gemm_splitk_reduce_s<T, 16>), dim3(nb), dim3(256), 0, s, g);
    else if (S == 8) MMSEG_LAUNCH((gemm_splitk_reduce_s<T, 8>), dim3(nb), dim3(256), 0, s, g);
    else if (S == 4) MMSEG_LAUNCH((gemm_splitk_reduce_s<T, 4>), dim3(nb), dim3(256), 0, s, g);
    else MMSEG_LAUNCH((gemm_splitk_reduce_s<T, 2>), dim3(nb), dim3(256), 0, s, g);
  } else {
    MMSEG_LAUNCH((gemm_splitk_reduce<T, MODE>), dim3(splitk_reduce_blocks<MODE>(g)), dim3(256), 0, s, g);
  }
  return mmseg::check_launch("gemm_splitk_reduce");
}

template <typename T, int MODE>
int launch_gemm(GemmArgs g, hipStream_t s) {
  if (g.nmean) {   // deferred InstanceNorm + ReLU of A: brick5 only (mmseg_conv3_norm_ok)
    MMSEG_REQUIRE(MODE == MODE_CONV3 && brick5_selected(g, (int)sizeof(T)),
                  "conv3 with a deferred norm needs the brick5 kernel for this shape (mmseg_conv3_norm_ok)");
    launch_brick5(g, s);
    return mmseg::check_launch("conv3_brick5_norm");
  }
  const int Cbig = g.Ncols >= 64;
  dim3 block(256);
  const int brick = knob("MMSEG_BRICK", 2);
  const Conv3Plan plan = MODE == MODE_CONV3 ? plan_conv3(g.M, g.Ncols, 8 << g.cpg_shift, g.D, g.H, g.W, g.lda, g.ldo,
                                                         (int)sizeof(T), g.grp_n > 0)
                                            : Conv3Plan{0, 0, 0, 0, 1, 32};
  MMSEG_REQUIRE(g.grp_n == 0 || (MODE == MODE_CONV3 && plan.kind == 2),
                "grouped conv: only the runtime-brick kernel takes per-group weights (small volumes)");
  if (plan.kind == 2) {
    const int nb = (g.M / (g.D * g.H * g.W)) * (g.D / plan.bz) * (g.H / plan.by) * (g.W / plan.bx);
    const int nchunk = gemm_nchunk(g);
    if (g.ksplit > nchunk) g.ksplit = nchunk;
    const int cps = (nchunk + g.ksplit - 1) / g.ksplit;
    g.ksplit = (nchunk + cps - 1) / cps;
    const dim3 grid(nb * ((g.Ncols + plan.bn - 1) / plan.bn) * g.ksplit);
    // compile-time bricks: 6 x 6 x 6 (the 12^3 / 6^3 levels) and 4 x 8 x 8 (the grouped 48^3 / 24^3 levels)
    const bool b666 = plan.bz == 6 && plan.by == 6 && plan.bx == 6;
    const bool b488 = plan.bz == 4 && plan.by == 8 && plan.bx == 8;
    // 32-bit offset halo staging (bf16 only, as conv3_brick2_kernel's B32; MMSEG_B32=0: the 64-bit staging)
    const bool rb32 = sizeof(T) == 2 && knob("MMSEG_B32", 1) && (long long)g.M * g.lda * (long long)sizeof(T) < (1LL << 31);
    if (plan.bn == 64) {
      if constexpr (sizeof(T) == 2) {
        MMSEG_TILE(g, "conv3_brickr_kernel<BN64>", 64);
        if (b666 && rb32)
          MMSEG_LAUNCH((conv3_brickr_kernel<T, 64, 6, 6, 6, 0, false, true>), grid, block, 0, s, g, 6, 6, 6, (long long*)nullptr);
        else if (b666)
          MMSEG_LAUNCH((conv3_brickr_kernel<T, 64, 6, 6, 6>), grid, block, 0, s, g, 6, 6, 6, (long long*)nullptr);
        else if (b488 && rb32)
          MMSEG_LAUNCH((conv3_brickr_kernel<T, 64, 4, 8, 8, 0, false, true>), grid, block, 0, s, g, 4, 8, 8, (long long*)nullptr);
        else if (b488)
          MMSEG_LAUNCH((conv3_brickr_kernel<T, 64, 4, 8, 8>), grid, block, 0, s, g, 4, 8, 8, (long long*)nullptr);
        else if (rb32)
          MMSEG_LAUNCH((conv3_brickr_kernel<T, 64, 0, 0, 0, 0, false, true>), grid, block, 0, s, g, plan.bz,
                             plan.by, plan.bx, (long long*)nullptr);
        else
          MMSEG_LAUNCH((conv3_brickr_kernel<T, 64>), grid, block, 0, s, g, plan.bz, plan.by, plan.bx, (long long*)nullptr);
      }
    } else if (b666) {
      // KW = 2: two waves per SIMD from an in-block split of the chunks (see the kernel); tap t + 1's fragments
      // read during tap t's MFMAs (PF: at 12^3 / 6^3 a CU holds one block; 5-10 % per launch, r04ab convbench)
      const bool kw2 = sizeof(T) == 2 && !g.stats && cps >= 2;
      MMSEG_TILE(g, kw2 ? "conv3_brickr_kernel<BN32,KW2>" : "conv3_brickr_kernel<BN32>", 32);
      bool done = false;
      if constexpr (sizeof(T) == 2) {   // (the fp32 form's two stage sets exceed the LDS)
        const dim3 b2(512);
        if (kw2 && rb32)
          MMSEG_LAUNCH((conv3_brickr_kernel<T, 32, 6, 6, 6, 0, true, true, 2>), grid, b2, 0, s, g, 6, 6, 6, nullptr);
        else if (kw2)
          MMSEG_LAUNCH((conv3_brickr_kernel<T, 32, 6, 6, 6, 0, true, false, 2>), grid, b2, 0, s, g, 6, 6, 6, nullptr);
        done = kw2;
      }
      if (done) {
      } else if (rb32)
        MMSEG_LAUNCH((conv3_brickr_kernel<T, 32, 6, 6, 6, 0, true, true>), grid, block, 0, s, g, 6, 6, 6, (long long*)nullptr);
      else
        MMSEG_LAUNCH((conv3_brickr_kernel<T, 32, 6, 6, 6>), grid, block, 0, s, g, 6, 6, 6, (long long*)nullptr);
    } else if (b488) {
      MMSEG_TILE(g, "conv3_brickr_kernel<BN32>", 32);
      if (rb32)
        MMSEG_LAUNCH((conv3_brickr_kernel<T, 32, 4, 8, 8, 0, false, true>), grid, block, 0, s, g, 4, 8, 8, (long long*)nullptr);
      else
        MMSEG_LAUNCH((conv3_brickr_kernel<T, 32, 4, 8, 8>), grid, block, 0, s, g, 4, 8, 8, (long long*)nullptr);
    } else {
      MMSEG_TILE(g, "conv3_brickr_kernel<BN32>", 32);
      if (rb32)
        MMSEG_LAUNCH((conv3_brickr_kernel<T, 32, 0, 0, 0, 0, false, true>), grid, block, 0, s, g, plan.bz,
                           plan.by, plan.bx, (long long*)nullptr);
      else
        MMSEG_LAUNCH((conv3_brickr_kernel<T, 32>), grid, block, 0, s, g, plan.bz, plan.by, plan.bx, (long long*)nullptr);
    }
    if (mmseg::check_launch("conv3_brickr")) return 1;
    if (g.ksplit > 1) return launch_splitk_reduce<T, MODE>(g, s);
    return 0;
  }
  if (plan.kind == 1 && g.ksplit == 1) {
    const int nb1 = (g.M / (g.D * g.H * g.W)) * (g.D / 4) * (g.H / B2_Y) * (g.W / B2_X);
    const int min_blocks = knob("MMSEG_BRICK2_MINBLK", 512);
    if constexpr (sizeof(T) == 2) {
      // 8-wave 8x8x8 brick with LDS-DMA staging (conv3_brick8_kernel)
      const int nb8 = nb1 / 2;   // 8-deep bricks
      // (BN64: one 64-column tile over >= 2 input chunks, where it measured faster than brick2 BN64 -- 48^3
      // 64->64 fwd / dgrad 61 -> 55.5 us, 128->64 fwd 111 -> 98 us; with one chunk, or two column tiles, it was
      // slower: profiles/r03c_brick8_convbench.txt)
      const int b8 = knob("MMSEG_BRICK8", 1);
      if (b8 && g.Ncols % 64 == 0 && (b8 == 2 || (g.Ncols == 64 && gemm_nchunk(g) >= 2)) && g.D % 8 == 0 &&
          g.H % 8 == 0 && g.W % 8 == 0 &&
          g.stats == nullptr && g.nmean == nullptr && g.inpart == nullptr && g.ldo % 8 == 0 &&
          (!g.out2 || g.ldo2 % 8 == 0) && (reinterpret_cast<uintptr_t>(g.out) & 15) == 0 &&
          nb8 * (g.Ncols / 64) >= knob("MMSEG_BRICK8_MINBLK", 256) &&
          (long long)g.M * g.lda * 2 < (1LL << 31) && (long long)((g.KG + 3) & ~3) * g.Cpad * 16 < (1LL << 31)) {
        MMSEG_TILE(g, "conv3_brick8_kernel<BN64>", 64);
        MMSEG_LAUNCH((conv3_brick8_kernel<64, 1>), dim3(nb8 * (g.Ncols / 64)), dim3(512), 0, s, g);
        return mmseg::check_launch("conv3_brick8");
      }
      if (b8 && g.Ncols == 32 && g.D % 16 == 0 && g.H % 8 == 0 && g.W % 8 == 0 &&
          g.stats == nullptr && g.nmean == nullptr && g.inpart == nullptr && g.ldo % 8 == 0 &&
          (!g.out2 || g.ldo2 % 8 == 0) && (reinterpret_cast<uintptr_t>(g.out) & 15) == 0 &&
          nb8 / 2 >= knob("MMSEG_BRICK8_MINBLK", 256) && (8 << g.cpg_shift) >= 64 &&
          (long long)g.M * g.lda * 2 < (1LL << 31) && (long long)((g.KG + 3) & ~3) * g.Cpad * 16 < (1LL << 31)) {
        MMSEG_TILE(g, "conv3_brick8_kernel<BN32>", 32);
        MMSEG_LAUNCH((conv3_brick8_kernel<32, 2>), dim3(nb8 / 2), dim3(512), 0, s, g);
        return mmseg::check_launch("conv3_brick8");
      }
    }
    // v3 is bf16 only: its fp32 instantiation (f32 16x16x4 MFMA with swapped operands) returned the first
    // row of each 4-row accumulator group in all four registers (tools/diag_b3.py); the fp32 parity path
    // keeps the v2 kernel.
    const bool v3 = sizeof(T) == 2 && g.stats == nullptr && (long long)g.M * g.lda * (long long)sizeof(T) < (1LL << 31);
    // persistent: at most one wave of resident blocks (2 per CU), each over a contiguous range of units
    const int maxblk = knob("MMSEG_BRICK3_BLOCKS", 512);
    // 32-bit offset halo staging (brick2 B32; bf16 only, see the runtime-brick branch)
    const bool b32 = sizeof(T) == 2 && knob("MMSEG_B32", 1) && (long long)g.M * g.lda * (long long)sizeof(T) < (1LL << 31);
    const bool wide = g.Ncols % 64 == 0 && nb1 * (g.Ncols / 64) >= min_blocks;
    // 48-column tiles also for multiples of 96 that are not of 64 (SwinUNETR's 96-column convs: two 48-column tiles
    // read the A halo twice, three 32-column brick3 tiles three times -- 128^3 96-column dgrad 0.74 ms at 706 TF/s
    // on brick3, r05c timer)
    const bool bn48 = g.Ncols % 32 != 0 || (g.Ncols % 96 == 0 && g.Ncols % 64 != 0 && g.stats == nullptr);
    if (bn48) {    // a multiple of 48 (plan_conv3)
      MMSEG_TILE(g, "conv3_brick2_kernel<BN48,ZW1>", 48);
      if (b32) {
        MMSEG_LAUNCH((conv3_brick2_kernel<T, 48, 1, false, true>), dim3(nb1 * (g.Ncols / 48)), block, 0, s, g);
        return mmseg::check_launch("conv3_brick2");
      }
      MMSEG_LAUNCH((conv3_brick2_kernel<T, 48, 1>), dim3(nb1 * (g.Ncols / 48)), block, 0, s, g);
    } else if (v3 && gemm_nchunk(g) == 1 && g.Ncols % 32 == 0 && !wide) {
      if constexpr (sizeof(T) == 2) {
        // one persistent block per CU, each over a contiguous brick range of one 32-column tile
        const int nt_n = g.Ncols / 32;
        const int per_nt = std::max(1, knob("MMSEG_BRICK4_BLOCKS", 256) / nt_n);
        const int upb = ceil_div(nb1, std::min(per_nt, nb1));
        const int bpn = ceil_div(nb1, upb);
        if (g.H % 4 == 0 && g.W % 16 == 0 && g.ldo % 8 == 0 && (reinterpret_cast<uintptr_t>(g.out) & 15) == 0) {
          launch_brick5(g, s);   // (16-B output stores)
        } else {
          MMSEG_TILE(g, "conv3_brick4_kernel<BN32>", 32);
          MMSEG_LAUNCH(conv3_brick4_kernel, dim3(bpn * nt_n), block, 0, s, g, upb, bpn);
        }
      }
    } else if (v3 && !wide) {
      const int units = nb1 * (g.Ncols / 32);
      const int upb = maxblk > 0 ? ceil_div(units, maxblk) : 1;
      MMSEG_TILE(g, "conv3_brick3_kernel<BN32>", 32);
      MMSEG_LAUNCH((conv3_brick3_kernel<T, 32>), dim3(ceil_div(units, upb)), block, 0, s, g, upb);
    } else if (wide) {
      // each tap's fragments read while the previous tap's MFMAs run (2 % on the 48^3 64-channel layers, r02)
      MMSEG_TILE(g, "conv3_brick2_kernel<BN64,ZW1>", 64);
      if (b32)
        MMSEG_LAUNCH((conv3_brick2_kernel<T, 64, 1, true, true>), dim3(nb1 * (g.Ncols / 64)), block, 0, s, g);
      else
        MMSEG_LAUNCH((conv3_brick2_kernel<T, 64, 1, true>), dim3(nb1 * (g.Ncols / 64)), block, 0, s, g);
    } else {
      MMSEG_TILE(g, "conv3_brick2_kernel<BN32,ZW1>", 32);
      MMSEG_LAUNCH((conv3_brick2_kernel<T, 32, 1>), dim3(nb1 * (g.Ncols / 32)), block, 0, s, g);
    }
    return mmseg::check_launch("conv3_brick2");
  }
  if (MODE == MODE_CONV3 && g.ksplit == 1 && brick == 1 && (8 << g.cpg_shift) % CK == 0 &&
      g.D % BRK_Z == 0 && g.H % BRK_Y == 0 && g.W % BRK_X == 0 && g.lda % 8 == 0) {
    const int nb = (g.M / (g.D * g.H * g.W)) * (g.D / BRK_Z) * (g.H / BRK_Y) * (g.W / BRK_X);
    const int bn = g.Ncols >= 64 ? 64 : 32;
    MMSEG_TILE(g, bn == 64 ? "conv3_brick_kernel<BN64>" : "conv3_brick_kernel<BN32>", bn);
    if (bn == 64) {
      MMSEG_LAUNCH((conv3_brick_kernel<T, 64>), dim3(nb * ceil_div(g.Ncols, 64)), block, 0, s, g);
    } else {
      MMSEG_LAUNCH((conv3_brick_kernel<T, 32>), dim3(nb * ceil_div(g.Ncols, 32)), block, 0, s, g);
    }
    return mmseg::check_launch("conv3_brick");
  }
  if (MODE == MODE_CONVT_FWD && g.Ncols % 256 == 0) {
    // BM=64, BN=256: a block writes all 8 taps x 32 (or a quarter of 8 x 128 ...) output channels of its 64 input
    // voxels, so each input row is read by one block instead of by Ncols / 64 column tiles
    MMSEG_TILE(g, "conv_gemm_kernel<convT_fwd,64x256>", 256);
    dim3 grid(ceil_div(g.M, 64) * (g.Ncols / 256) * g.ksplit);
    MMSEG_LAUNCH((conv_gemm_kernel<T, MODE, 1, 4, 4, 4>), grid, block, 0, s, g);
    if (mmseg::check_launch("conv_gemm")) return 1;
    if (g.ksplit > 1) return launch_splitk_reduce<T, MODE>(g, s);
    return 0;
  }
  if (MODE == MODE_POINT && g.ksplit == 1 && g.Ncols > 128 && g.Ncols <= 192 && g.Cpad >= 192) {
    // BM=64, BN=192: SwinUNETR's 144 / 192-column token linears (qkv, MLP fc1, fc2's data gradient) with every A
    // row read by one block -- 128x64 tiles re-read each K-wide row from L2 / HBM once per column tile
    if constexpr (MODE == MODE_POINT) {
      MMSEG_TILE(g, "conv_gemm_kernel<point,64x192>", 192);
      dim3 grid(ceil_div(g.M, 64));
      MMSEG_LAUNCH((conv_gemm_kernel<T, MODE, 1, 4, 4, 3>), grid, block, 0, s, g);
    }
  } else if (MODE == MODE_POINT && g.ksplit == 1 && g.Ncols > 64 && g.Ncols <= 128 && g.Ncols % 96 != 0) {
    // BM=64, BN=128: 128-column outputs (the residual 1x1 convs' data gradients written as whole 96-of-128 rows)
    // in one column tile -- the 128x64 tile read every A row twice (the 128^3 decoder's: 295 us, r06k)
    if constexpr (MODE == MODE_POINT) {
      MMSEG_TILE(g, "conv_gemm_kernel<point,64x128>", 128);
      dim3 grid(ceil_div(g.M, 64));
      MMSEG_LAUNCH((conv_gemm_kernel<T, MODE, 1, 4, 4, 2>), grid, block, 0, s, g);
    }
  } else if (MODE == MODE_POINT && g.ksplit == 1 && g.Ncols > 32 && g.Ncols <= 48 && g.Ncols % 16 == 0) {
    // BM=128, BN=48: the 48-column token linears / 1x1 convs (feature_size 48) in one column tile (BN=32 took two)
    if constexpr (MODE == MODE_POINT) {
      MMSEG_TILE(g, "conv_gemm_kernel<point,128x48>", 48);
      dim3 grid(ceil_div(g.M, 128));
      MMSEG_LAUNCH((conv_gemm_kernel<T, MODE, 4, 1, 2, 3>), grid, block, 0, s, g);
    }
  } else if (MODE == MODE_POINT && g.Ncols % 96 == 0 && g.Ncols % 64 != 0) {
    // BM=128, BN=96: the 96 / 288 / 480-column 1x1 GEMMs (SwinUNETR's 96-channel stage, the 96 -> 48 residual
    // conv's data gradient) in whole tiles -- BN=64 left a half-empty last column tile that re-read every A row
    if constexpr (MODE == MODE_POINT) {
      MMSEG_TILE(g, "conv_gemm_kernel<point,128x96>", 96);
      dim3 grid(ceil_div(g.M, 128) * (g.Ncols / 96) * g.ksplit);
      MMSEG_LAUNCH((conv_gemm_kernel<T, MODE, 2, 2, 4, 3>), grid, block, 0, s, g);
    }
  } else if (!Cbig) {
    // BM=128, BN=32
    static const char* nm[4] = {"conv_gemm_kernel<conv3,128x32>", "conv_gemm_kernel<point,128x32>",
                                "conv_gemm_kernel<convT_fwd,128x32>", "conv_gemm_kernel<convT_dgrad,128x32>"};
    MMSEG_TILE(g, nm[MODE], 32);
    dim3 grid(ceil_div(g.M, 128) * ceil_div(g.Ncols, 32) * g.ksplit);
    MMSEG_LAUNCH((conv_gemm_kernel<T, MODE, 4, 1, 2, 2>), grid, block, 0, s, g);
  } else {
    // BM=128, BN=64
    static const char* nm[4] = {"conv_gemm_kernel<conv3,128x64>", "conv_gemm_kernel<point,128x64>",
                                "conv_gemm_kernel<convT_fwd,128x64>", "conv_gemm_kernel<convT_dgrad,128x64>"};
    MMSEG_TILE(g, nm[MODE], 64);
    dim3 grid(ceil_div(g.M, 128) * ceil_div(g.Ncols, 64) * g.ksplit);
    MMSEG_LAUNCH((conv_gemm_kernel<T, MODE, 2, 2, 4, 2>), grid, block, 0, s, g);
  }
  if (mmseg::check_launch("conv_gemm")) return 1;
  if (g.ksplit > 1) return launch_splitk_reduce<T, MODE>(g, s);
  return 0;
}

template <typename T>
int launch_gemm_mode(GemmArgs g, int mode, hipStream_t s) {
  switch (mode) {
    case MODE_CONV3: return launch_gemm<T, MODE_CONV3>(g, s);
    case MODE_POINT: return launch_gemm<T, MODE_POINT>(g, s);
    case MODE_CONVT_FWD: return launch_gemm<T, MODE_CONVT_FWD>(g, s);
    case MODE_CONVT_DGRAD: return launch_gemm<T, MODE_CONVT_DGRAD>(g, s);
  }
  mmseg::set_error("bad gemm mode %d", mode);
  return 1;
}

// The LDS-DMA weight-gradient kernel's row tile (4 = 64 co, 2 = 32 co) when it takes this CONV3 brick2 launch,
// else 0: bf16, byte offsets of both tensors within 31 bits (the deferred-norm variant keeps register staging by
// default: its in-place LDS pass and extra barrier cost more than the DMA saves, 0.651 -> 0.682 ms/step for the
// 32-co family)
bool wgrad_co64(int Ca, long long V, int kind);

int wgrad_dma_mt(const WgradArgs& g, int elem_bytes) {
  const bool dma = elem_bytes == 2 && g.brick == 2 && knob("MMSEG_WGRAD_DMA", 1) && g.nmean == nullptr &&
                   g.V * g.lda * 2 < (1LL << 31) &&
                   g.V * g.ldb * 2 < (1LL << 31) && (g.lda % 8) == 0 && (g.ldb % 8) == 0;
  return dma ? (wgrad_co64(g.Ca, g.V, 2) ? 4 : 2) : 0;
}

// the row-slab weight gradient (wgrad_row_kernel) takes the shape: bf16 3^3, 32 output channels, W % 32 == 0,
// H % 4 == 0, split partials (no direct gradient, no groups, no padded rows), 32-bit DMA offsets
// rows per step: 6 where H allows (r06c, 96^3 B=2: 32 -> 32 deferred norm 128.6 -> 113.6 us, 64 -> 32 196 -> 179 us
// against 4 rows; five ring slots or s_setprio for waves 6..11 measured no change), else 4
bool wgrad_row_ok(const WgradArgs& g, int elem_bytes) {
  return elem_bytes == 2 && knob("MMSEG_WGRAD_ROW", 1) && g.brick == 2 && g.Ca == 32 && g.W % 32 == 0 &&
         g.H % 4 == 0 && (8 << g.cpg_shift) % CK == 0 && g.groups == 0 && !g.pad16 && g.ksplit > 1 &&
         g.V * g.lda * 2 < (1LL << 31) && g.V * g.ldb * 2 < (1LL << 31) && g.lda % 8 == 0 && g.ldb % 8 == 0 &&
         g.V / ((long long)g.D * g.H * g.W) <= WROW_MAXN;
}

template <typename T, int MODE>
int launch_wgrad(WgradArgs g, hipStream_t s) {
  g.dbg = 0;   // (the timing probes of the brick weight-gradient kernels: 1 no loads, 2 no MFMA; diagnostics only)
  dim3 block(256);
  if constexpr (sizeof(T) == 2) {
    if (MODE == MODE_CONV3 && g.brick == 3) {
      const WBrick wb = plan_wgrad_brickr(g.D, g.H, g.W);
      const bool b366 = wb.bz == 3 && wb.by == 6 && wb.bx == 6;
      const bool b448 = wb.bz == 4 && wb.by == 4 && wb.bx == 8;   // grouped 48^3 / 24^3
      if (wgrad_co64(g.Ca, g.V, 3)) {
        dim3 grid(wgrad_nchunk(g.cpg_shift, g.kchunks) * (g.Ca / 64) * g.ksplit);
        // (the compile-time bricks under their rocprofv3 family names, tools/rocprof_families.py)
        mmseg::note_kernel(b366 ? "wgrad_brickr_kernel<CO64,V3>" : b448 ? "wgrad_brickr_kernel<CO64,B448>"
                                                                         : "wgrad_brickr_kernel<CO64>");
        if (b366)
          MMSEG_LAUNCH((wgrad_brickr_kernel<T, 4, 3, 6, 6>), grid, dim3(512), 0, s, g, 3, 6, 6);
        else if (b448)
          MMSEG_LAUNCH((wgrad_brickr_kernel<T, 4, 4, 4, 8>), grid, dim3(512), 0, s, g, 4, 4, 8);
        else
          MMSEG_LAUNCH((wgrad_brickr_kernel<T, 4>), grid, dim3(512), 0, s, g, wb.bz, wb.by, wb.bx);
      } else {
        dim3 grid(wgrad_nchunk(g.cpg_shift, g.kchunks) * (g.Ca / 32) * g.ksplit);
        mmseg::note_kernel(b366 ? "wgrad_brickr_kernel<CO32,V3>" : b448 ? "wgrad_brickr_kernel<CO32,B448>"
                                                                         : "wgrad_brickr_kernel<CO32>");
        if (b366)
          MMSEG_LAUNCH((wgrad_brickr_kernel<T, 2, 3, 6, 6>), grid, dim3(512), 0, s, g, 3, 6, 6);
        else if (b448)
          MMSEG_LAUNCH((wgrad_brickr_kernel<T, 2, 4, 4, 8>), grid, dim3(512), 0, s, g, 4, 4, 8);
        else
          MMSEG_LAUNCH((wgrad_brickr_kernel<T, 2>), grid, dim3(512), 0, s, g, wb.bz, wb.by, wb.bx);
      }
      return mmseg::check_launch("wgrad_brickr");
    }
    if (MODE == MODE_CONV3 && g.brick == 2 && wgrad_row_ok(g, (int)sizeof(T))) {
      MMSEG_REQUIRE(g.frag, "wgrad_row: fragment-native partials only");
      const dim3 grid(wgrad_nchunk(g.cpg_shift, g.kchunks) * g.ksplit);
      auto run = [&](auto normc) {
        constexpr bool NRM = decltype(normc)::value;
        if (g.H % 6 == 0)
          MMSEG_LAUNCH((wgrad_row_kernel<NRM, 6>), grid, dim3(768), 0, s, g);
        else
          MMSEG_LAUNCH((wgrad_row_kernel<NRM, 4>), grid, dim3(768), 0, s, g);
      };
      if (g.nmean) {
        mmseg::note_kernel("wgrad_row_kernel<CO32,NORM>");
        run(std::true_type{});
      } else {
        mmseg::note_kernel("wgrad_row_kernel<CO32>");
        run(std::false_type{});
      }
      return mmseg::check_launch("wgrad_row");
    }
    if (MODE == MODE_CONV3 && g.brick == 2) {
      if (const int mt = wgrad_dma_mt(g, (int)sizeof(T))) {
        dim3 grid(wgrad_nchunk(g.cpg_shift, g.kchunks) * (g.Ca / (16 * mt)) * g.ksplit);
        if (mt == 4) {
          mmseg::note_kernel("wgrad_dma_kernel<CO64>");
          // 48 real rows of 64 (SwinUNETR's 48-channel levels): three row tiles, room for the pipelined multiply
          if (g.pad16 && g.Ca == 64)
            MMSEG_LAUNCH((wgrad_dma_kernel<4, false, 3, true, 3>), grid, dim3(512), 0, s, g);
          else   // (fragment prefetch two steps ahead spills at 64 co: 59.5 -> 72.3 us)
            MMSEG_LAUNCH((wgrad_dma_kernel<4>), grid, dim3(512), 0, s, g);
        } else {
          mmseg::note_kernel("wgrad_dma_kernel<CO32>");
          MMSEG_LAUNCH((wgrad_dma_kernel<2, false, 3, true>), grid, dim3(512), 0, s, g);
        }
        return mmseg::check_launch("wgrad_dma");
      }
      if (wgrad_co64(g.Ca, g.V, 2)) {
        dim3 grid(wgrad_nchunk(g.cpg_shift, g.kchunks) * (g.Ca / 64) * g.ksplit);
        mmseg::note_kernel("wgrad_brick2_kernel<CO64,V3>");
        if (g.nmean)
          MMSEG_LAUNCH((wgrad_brick2_kernel<T, 4, 3, true>), grid, dim3(512), 0, s, g);
        else
          MMSEG_LAUNCH((wgrad_brick2_kernel<T, 4, 3>), grid, dim3(512), 0, s, g);
      } else {
        // (fragment reads software-pipelined, r05: the deferred-norm 96^3 layers 136 -> 125 us before wgrad_row)
        dim3 grid(wgrad_nchunk(g.cpg_shift, g.kchunks) * (g.Ca / 32) * g.ksplit);
        mmseg::note_kernel("wgrad_brick2_kernel<CO32,V3>");
        if (g.nmean)
          MMSEG_LAUNCH((wgrad_brick2_kernel<T, 2, 3, true, true>), grid, dim3(512), 0, s, g);
        else
          MMSEG_LAUNCH((wgrad_brick2_kernel<T, 2, 3, false, true>), grid, dim3(512), 0, s, g);
      }
      return mmseg::check_launch("wgrad_brick2");
    }
  }
  if (MODE == MODE_CONV3 && g.brick) {
    dim3 grid(wgrad_nchunk(g.cpg_shift, g.kchunks) * (g.Ca / 32) * g.ksplit);
    mmseg::note_kernel("wgrad_brick_kernel");
    MMSEG_LAUNCH((wgrad_brick_kernel<T>), grid, block, 0, s, g);
    return mmseg::check_launch("wgrad_brick");
  }
  static const char* nm[4] = {"wgrad_kernel<conv3>", "wgrad_kernel<point>", "wgrad_kernel<convT_fwd>",
                              "wgrad_kernel<convT_dgrad>"};
  mmseg::note_kernel(nm[MODE]);
  // 1x1 weight gradients take 64-row tiles whatever the row count (rows past Ca are masked): every row tile re-reads
  // the whole B operand (x), and these launches are HBM-bound -- 48 / 144-row layers read x once / three times
  // instead of twice / five times with 32-row tiles
  if (g.Ca % 64 == 0 || MODE == MODE_POINT) {
    dim3 grid(ceil_div(g.Ncols, 64) * ceil_div(g.Ca, 64) * g.ksplit);
    MMSEG_LAUNCH((wgrad_kernel<T, MODE, 2, 2, 2, 2, 64>), grid, block, 0, s, g);
  } else {
    dim3 grid(ceil_div(g.Ncols, 64) * ceil_div(g.Ca, 32) * g.ksplit);
    MMSEG_LAUNCH((wgrad_kernel<T, MODE, 1, 4, 2, 1, 64>), grid, block, 0, s, g);
  }
  return mmseg::check_launch("wgrad");
}

// 0: generic wgrad_kernel, 1: wgrad_brick_kernel (32 co), 2: wgrad_brick2_kernel (64 / 32 co),
// 3: wgrad_brickr_kernel (runtime brick, small volumes).
// (v2 / runtime brick are bf16 only: their two fp32 stage buffers would not fit in LDS)
int wgrad_brick_ok(int Ca, int cpg_shift, int D, int H, int W, int lda, int ldb, int dtype, bool force_r = false) {
  const int k = knob("MMSEG_WGRAD_BRICK", 2);
  if (!(k && Ca % 32 == 0 && (8 << cpg_shift) % CK == 0 && lda % 8 == 0 && ldb % 8 == 0)) return 0;
  if (force_r)   // grouped launches: only the runtime-brick weight gradient splits by sample group
    return (k >= 2 && dtype == MMSEG_BF16 && plan_wgrad_brickr(D, H, W).bz) ? 3 : 0;
  if (D % BRK_Z == 0 && H % BRK_Y == 0 && W % BRK_X == 0)
    return (k >= 2 && dtype == MMSEG_BF16) ? 2 : 1;
  if (k >= 2 && dtype == MMSEG_BF16 && plan_wgrad_brickr(D, H, W).bz) return 3;
  return 0;
}

// Split count of the CONV3 brick wgrad: enough blocks to fill the chip, capped by
// the caller's workspace (cap) and by one brick per split.
// 64-co row tiles for the brick weight-gradient kernels (kind 2: brick2 / LDS-DMA, 3: runtime brick), else 32-co.
// A block's split partial is its whole tile, so at small volumes -- where the ~256 resident blocks each see a
// few bricks -- the partials outweigh the inputs (24^3: 54 MB written and re-read per launch against 35-65 MB
// of input); 32-co tiles halve them at the price of reading the halo once per row tile.  Below V voxels
// a threshold the 32-co tiles were tried below (r04: equal or slower at 24^3), so 64-co tiles throughout.
bool wgrad_co64(int Ca, long long V, int kind) { return Ca % 64 == 0; }

int brick_wgrad_splits(long long V, int cap, int Ca, int cpg_shift, int kind, int D, int H, int W,
                       int kchunks = 0) {
  const int nchunk = wgrad_nchunk(cpg_shift, kchunks);
  const int tiles = nchunk * (Ca / ((kind >= 2 && wgrad_co64(Ca, V, kind)) ? 64 : 32));
  // v2 / runtime-brick kernels: one wave of resident blocks (256 CUs x blocks per CU: 2 for the 32-co brick2
  // kernel, 1 for the 64-co and runtime-brick kernels, whose stage buffers take > 80 KB of LDS), never more:
  // a partial second wave of 512-thread blocks costs a whole block time.
  long long ks;
  if (kind >= 2) {
    // (256 slots for the runtime-brick kernel too: 128 / 384 / 512 measured +0.04..0.15 ms per step, r04ah)
    ks = 256LL / tiles;
  } else {
    ks = (1024 + tiles - 1) / tiles;
  }
  if (ks > cap) ks = cap;
  long long nbrick = V / 128;
  if (kind == 3) {
    const WBrick wb = plan_wgrad_brickr(D, H, W);
    nbrick = V / (wb.bz * wb.by * wb.bx);
    // at least 4 bricks per split: at 6^3 (4 bricks) one split writes the gradient directly; two splits moved 2x
    // the 28 MB fp32 gradient of a 512->512 layer through partials and a reduce (41 -> 24 us, r02 convbench)
    const long long minb = 4;
    if (ks > nbrick / minb) ks = nbrick / minb;
  }
  if (ks > nbrick) ks = nbrick;
  if (ks < 1) ks = 1;
  const long long bpk = (nbrick + ks - 1) / ks;
  return (int)((nbrick + bpk - 1) / bpk);
}


int mmseg_wgrad_splits_impl(long long V, int ksplit) {
  long long vps = ((V + ksplit - 1) / ksplit + 63) / 64 * 64;
  return (int)((V + vps - 1) / vps);
}

// Real 32-channel chunks of a channel-padded x (Ci < Cip), 0 = all (the brick wgrad kernels skip the rest; the
// split reduction never reads the skipped columns' partials into the gradient).
int wgrad_kchunks(int Cip, int Ci) { return Ci < Cip ? (Ci + 31) / 32 : 0; }

// A single-split brick weight gradient writes the torch-layout gradient [co][ci][27] itself when its input
// channels are unpadded, or padded past whole real 32-channel chunks (Ci % 32 == 0: SwinUNETR's 768 of 1024): the
// kernel computes only the real chunks (wgrad_kchunks), whose rows then land at pitch 27 Ci (WgradArgs::grad_ld)
// -- no partial, no relayout reduce.
bool wgrad_direct_ok(int Cip, int Ci) {
  return Ci == Cip || (Ci % 32 == 0 && wgrad_kchunks(Cip, Ci) == Ci / 32);
}

// CONV3 weight-gradient plan (mmseg_conv3_wgrad): kernel kind (wgrad_brick_ok), split count, whether the
// kernel writes the torch-layout gradient itself (brick2 / brickr, one split, unpadded input channels),
// and the workspace (floats) of the split partials + bias partials otherwise.
struct Conv3WgradPlan {
  int kind, ksplit, direct;
  long long ws;
};

Conv3WgradPlan plan_conv3_wgrad(long long V, int Co, int Cip, int Ci, int cpg_shift, int D, int H, int W, int lda,
                                int ldb, int dtype, long long ws_cap, bool force_r = false) {
  Conv3WgradPlan p{0, 1, 0, 0};
  const long long ncols = 27LL * Cip;
  const long long per_split = (long long)Co * ncols + Co;
  int cap = (int)(ws_cap / per_split);
  if (cap < 1) cap = 1;
  p.kind = wgrad_brick_ok(Co, cpg_shift, D, H, W, lda, ldb, dtype, force_r);
  if (p.kind) {
    p.ksplit = brick_wgrad_splits(V, cap, Co, cpg_shift, p.kind, D, H, W, wgrad_kchunks(Cip, Ci));
  } else {
    const int bn = 64;
    const long long tiles = ((ncols + bn - 1) / bn) * ((Co + (Co % 64 == 0 ? 63 : 31)) / (Co % 64 == 0 ? 64 : 32));
    long long want = (1024 + tiles - 1) / tiles;
    if (want > V / 512) want = V / 512;
    if (want > cap) want = cap;
    if (want < 1) want = 1;
    p.ksplit = mmseg_wgrad_splits_impl(V, (int)want);
  }
  p.direct = p.kind >= 2 && p.ksplit == 1 && wgrad_direct_ok(Cip, Ci);
  p.ws = p.direct ? 0 : p.ksplit * per_split;
  return p;
}

// split slices S of a reduce: about 8 split loads per thread, the slice sums a pairwise
// LDS tree; small gradients over many splits (the stem: 1,056 values x 1,024 splits) take more slices until the
// grid fills the chip, down to 2 loads per thread (S = 64 left it at 66 blocks, 12.8 us for 4 MB)
int wred_slices(const WReduceArgs& g) {
  const int ksplit = g.ksplit;
  const long long total = (long long)g.Ca * g.Ncols + (g.bias_part ? g.Ca : 0);
  int S = 1;
  while (S < 64 && ksplit / (2 * S) >= 8) S *= 2;
  while (S < 256 && (total * S + 1023) / 1024 < 512 && ksplit / (2 * S) >= 2) S *= 2;
  return S;
}

// reduces deferred by conv3_wgrad_impl (phase bit 4) until mmseg_wgrad_reduce_flush
struct PendingWred {
  WReduceArgs r;
  int groups;
  void* stream;
};
std::vector<PendingWred> g_wred_pending;
extern "C" int mmseg_wgrad_reduce_flush(void* stream);

// Queue a deferred reduce (summed by the next mmseg_wgrad_reduce_flush on its stream).  (Flushing early, once
// 60-240 MB of partials are queued so they are re-read from the Infinity Cache, measured +0.03..0.12 ms: r04.)
int wred_push(const WReduceArgs& r, int groups, void* stream) {
  // a queued reduce reads its partials when the queue is flushed: a second weight-gradient kernel into the same
  // partial buffer before that would have overwritten them (the engine flushes first: Runtime.own_part)
  for (const auto& e : g_wred_pending)
    if (e.stream == stream && (e.r.part == r.part || (r.bias_part && e.r.bias_part == r.bias_part))) {
      mmseg::set_error("deferred weight-gradient reduce: its partial buffer is already queued on this stream "
                       "(flush the queue before reusing it)");
      return -1;
    }
  g_wred_pending.push_back({r, groups, stream});
  return 0;
}

int launch_wgrad_reduce(WReduceArgs g, void* stream, int groups = 1) {
  const long long total = (long long)g.Ca * g.Ncols + (g.bias_part ? g.Ca : 0);
  hipStream_t s = (hipStream_t)stream;
  const int S = wred_slices(g);
#define MMSEG_WRED(SS, NB)                                                                             \
  case SS:                                                                                             \
    MMSEG_LAUNCH((wgrad_reduce_kernel<SS, 4>), dim3(ceil_div(total, NB), groups), dim3(256), 0, s, g);  \
    break;
  switch (S) {
    MMSEG_WRED(256, 4)
    MMSEG_WRED(128, 8)
    MMSEG_WRED(64, 16)
    MMSEG_WRED(32, 32)
    MMSEG_WRED(16, 64)
    MMSEG_WRED(8, 128)
    MMSEG_WRED(4, 256)
    MMSEG_WRED(2, 512)
    default:
      MMSEG_WRED(1, 1024)
  }
#undef MMSEG_WRED
  return mmseg::check_launch("wgrad_reduce");
}

}  // namespace

// e4m3 B-operand image of a 3^3 conv for brick6 F8 ([KGp][Cpad][8] bytes, the bf16 image's geometry): one block
// per output channel: s = 448 / max |w[co]| (1 for an all-zero row; 448 = e4m3fn's largest finite value), the
// entries w[co][ci][tap] * s rounded to e4m3 (v_cvt_pk_fp8_f32: round to nearest even), wdq[co] = 1 / s.
__global__ __launch_bounds__(256) void pack_conv3_fp8_kernel(const float* __restrict__ w, int Ci, int Cip, int Cpad,
                                                             unsigned char* __restrict__ dst, float* __restrict__ wdq) {
  const int co = blockIdx.x, tid = threadIdx.x;
  const int n = Ci * 27;
  const float* wr = w + (long long)co * n;
  float m = 0.f;
  for (int e = tid; e < n; e += 256) m = fmaxf(m, fabsf(wr[e]));
  __shared__ float red[4];
  m = fmaxf(m, __shfl_xor(m, 1, 64));
#pragma unroll
  for (int o = 2; o < 64; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((tid & 63) == 0) red[tid >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float sc = m > 0.f ? 448.f / m : 1.f;
  if (tid == 0) wdq[co] = 1.f / sc;
  for (int e = tid; e < n; e += 256) {
    const int ci = e / 27, tap = e - ci * 27;
    const int kgi = tap * (Cip / 8) + ci / 8;
    const int v = __builtin_amdgcn_cvt_pk_fp8_f32(wr[e] * sc, 0.f, 0, false);
    dst[((long long)kgi * Cpad + co) * 8 + (ci & 7)] = (unsigned char)(v & 0xff);
  }
}

// =================================================================== C ABI
extern "C" {

// Pack fp32 torch-layout weights into the MFMA B-operand layout [KGp][Cpad][8].
int mmseg_pack_weight(const float* w, void* dst, int mode, int Co, int Ci, int Cip, int KG, int KGp, int Cpad,
                      int dtype, void* stream) {
  PackArgs g{w, dst, Co, Ci, Cip, KG, KGp, Cpad};
  long long total = (long long)KGp * Cpad * 8;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMSEG_BF16)
    MMSEG_LAUNCH(pack_weight_kernel<bf16_t>, dim3(ceil_div(total, 256)), dim3(256), 0, s, g, mode);
  else
    MMSEG_LAUNCH(pack_weight_kernel<float>, dim3(ceil_div(total, 256)), dim3(256), 0, s, g, mode);
  return mmseg::check_launch("pack_weight");
}

int mmseg_pack3_desc_bytes(void) { return (int)sizeof(Pack3Desc); }

int mmseg_adamw_pack_desc_bytes(void) { return (int)sizeof(AdamPackDesc); }

static int adamw_pack_launch(float* p, const float* g, float* m, float* v, const void* descs, int n, int nblocks,
                             const AdamHyper& hv, const AdamHyper* hp, const float* skip, int dtype,
                             hipStream_t s) {
  MMSEG_REQUIRE(n >= 1 && nblocks >= 1 && descs != nullptr, "adamw_pack: a descriptor table (Packer.adam_table)");
  MMSEG_REQUIRE(((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(m) |
                  reinterpret_cast<uintptr_t>(v)) & 15) == 0, "adamw_pack: p, g, m, v must be 16-B aligned");
  if (dtype == MMSEG_BF16)
    MMSEG_LAUNCH(adamw_pack_kernel<bf16_t>, dim3(nblocks), dim3(256), 0, s, p, g, m, v, (const AdamPackDesc*)descs,
                 n, hv, hp, skip);
  else
    MMSEG_LAUNCH(adamw_pack_kernel<float>, dim3(nblocks), dim3(256), 0, s, p, g, m, v, (const AdamPackDesc*)descs,
                 n, hv, hp, skip);
  return mmseg::check_launch("adamw_pack");
}

// descs: device array of n AdamPackDesc sorted by block_begin, nblocks blocks in all (Packer.adam_table); the
// step's hyper-parameters by value (as mmseg_adamw) or as the 8 device floats of mmseg_adamw_hyper (as
// mmseg_adamw_dev); skip as there.  p / g / m / v: the flat arenas, 16-B aligned.
int mmseg_adamw_pack(float* p, const float* g, float* m, float* v, const void* descs, int n, int nblocks, float lr,
                     float beta1, float beta2, float eps, float wd, int step, const float* skip, int dtype,
                     void* stream) {
  MMSEG_REQUIRE(step >= 1, "adamw_pack: step counts from 1");
  return adamw_pack_launch(p, g, m, v, descs, n, nblocks, adamw_hyper(lr, beta1, beta2, eps, wd, step), nullptr, skip,
                           dtype, (hipStream_t)stream);
}

int mmseg_adamw_pack_dev(float* p, const float* g, float* m, float* v, const void* descs, int n, int nblocks,
                         const float* hyper, const float* skip, int dtype, void* stream) {
  MMSEG_REQUIRE(hyper != nullptr, "adamw_pack_dev: hyper (8 device floats from mmseg_adamw_hyper) required");
  return adamw_pack_launch(p, g, m, v, descs, n, nblocks, AdamHyper{}, reinterpret_cast<const AdamHyper*>(hyper),
                           skip, dtype, (hipStream_t)stream);
}

#ifdef MMSEG_TIMING_PROBES
// probe builds only (tools/convbench.py --probe): buffer of 8 * PROBE_NB + 32 * 16 * 64 longs, or null to stop
int mmseg_probe_set(long long* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_probe), &buf, sizeof(buf)) == hipSuccess ? 0 : 1;
}
#endif

// descs: device array of n Pack3Desc sorted by block_begin; nblocks = total blocks
// (sum over layers of Co/8 * ceil(Ci/32)).  The images must be zero-initialised once.
int mmseg_pack_conv3_batched(const void* descs, int n, int nblocks, int dtype, void* stream) {
  MMSEG_REQUIRE(n >= 1 && nblocks >= 1, "pack_conv3_batched: empty table");
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMSEG_BF16)
    MMSEG_LAUNCH(pack_conv3_batched_kernel<bf16_t>, dim3(nblocks), dim3(256), 0, s, (const Pack3Desc*)descs, n);
  else
    MMSEG_LAUNCH(pack_conv3_batched_kernel<float>, dim3(nblocks), dim3(256), 0, s, (const Pack3Desc*)descs, n);
  return mmseg::check_launch("pack_conv3_batched");
}

// descs: device array of n PackDesc (64 B each, see mmseg_pack_desc_bytes); total = sum of KGp*Cpad*8.
int mmseg_pack_desc_bytes(void) { return (int)sizeof(PackDesc); }

int mmseg_pack_weights_batched(const void* descs, int n, long long total, int dtype, void* stream) {
  MMSEG_REQUIRE(n >= 1, "pack_weights_batched: n >= 1");
  hipStream_t s = (hipStream_t)stream;
  long long blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (dtype == MMSEG_BF16)
    MMSEG_LAUNCH(pack_weight_batched_kernel<bf16_t>, dim3((int)blocks), dim3(256), 0, s, (const PackDesc*)descs,
                       n, total);
  else
    MMSEG_LAUNCH(pack_weight_batched_kernel<float>, dim3((int)blocks), dim3(256), 0, s, (const PackDesc*)descs,
                       n, total);
  return mmseg::check_launch("pack_weights_batched");
}

// Generic implicit-GEMM: conv3 fwd / dgrad, 1x1, convT fwd / dgrad.
// Bricks per sample whose InstanceNorm partials the CONV3 kernel for this shape
// can emit from its epilogue (mmseg_conv_gemm_stats), or 0 when it cannot
// (gather GEMM, split-K).  Every brick holds V / (bricks per sample) voxels.
// The brick epilogues' fused statistics measured no net gain against the statistics pass (bench r01 q11; the
// grouped form equal per step, r04ad), so no shape offers them: 0 for every shape (the ABI entry stays).
int mmseg_conv3_stats_bricks(int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H, int W, int lda, int ldo,
                             int dtype) {
  return 0;
}

int mmseg_conv_gemm_stats(const void* a, int lda, const void* wpacked, const float* bias, void* out, int ldo,
                          float* splitk_ws, int mode, int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H,
                          int W, int ksplit, float* stats_part, int dtype, void* stream);

int mmseg_conv_gemm(const void* a, int lda, const void* wpacked, const float* bias, void* out, int ldo,
                    float* splitk_ws, int mode, int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H, int W,
                    int ksplit, int dtype, void* stream) {
  return mmseg_conv_gemm_stats(a, lda, wpacked, bias, out, ldo, splitk_ws, mode, M, Ncols, Cpad, KG, cpg_shift, D, H,
                               W, ksplit, nullptr, dtype, stream);
}

int mmseg_conv_gemm_ex(const void* a, int lda, const void* wpacked, const float* bias, void* out, int ldo,
                       float* splitk_ws, int mode, int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H,
                       int W, int ksplit, float* stats_part, int cin_real, int dtype, void* stream);

// mmseg_conv_gemm + per-brick InstanceNorm partials of the output (stats_part:
// [N][bricks per sample][Ncols][2] floats, see mmseg_conv3_stats_bricks).
int mmseg_conv_gemm_stats(const void* a, int lda, const void* wpacked, const float* bias, void* out, int ldo,
                          float* splitk_ws, int mode, int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H,
                          int W, int ksplit, float* stats_part, int dtype, void* stream) {
  return mmseg_conv_gemm_ex(a, lda, wpacked, bias, out, ldo, splitk_ws, mode, M, Ncols, Cpad, KG, cpg_shift, D, H, W,
                            ksplit, stats_part, 0, dtype, stream);
}

// mmseg_conv_gemm_stats for an A source whose channels past cin_real are padding (zero weights): the CONV3
// brick kernels skip the 32-channel chunks wholly past cin_real.  cin_real = 0: every channel is real.
int conv_gemm_impl(const void* a, int lda, const void* wpacked, const float* bias, void* out, int ldo, void* out2,
                   int ldo2, int split, float* splitk_ws, int mode, int M, int Ncols, int Cpad, int KG, int cpg_shift,
                   int D, int H, int W, int ksplit, float* stats_part, int cin_real, int dtype, void* stream,
                   int groups = 1, long long w_gstride = 0, int b_gstride = 0, const void* res = nullptr,
                   int ldres = 0, int zcols = 0);
int mmseg_conv3_group_stats_bricks(int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H, int W, int lda,
                                   int ldo, int dtype);

// mmseg_conv_gemm_group + the per-brick InstanceNorm partials of the output (stats_part [M / (D H W)]
// [mmseg_conv3_group_stats_bricks()][Ncols][2], (mean, M2) per brick; mmseg_instnorm_stats_bricks merges them)
// from the runtime-brick kernel's epilogue -- the grouped 48^3 / 24^3 levels' statistics without a pass over
// the conv output.
int mmseg_conv_gemm_group_stats(const void* a, int lda, const void* wpacked, const float* bias, void* out, int ldo,
                                int mode, int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H, int W,
                                int cin_real, int groups, long long w_gstride, int b_gstride, float* stats_part,
                                int dtype, void* stream) {
  MMSEG_REQUIRE(mode == MODE_CONV3 && groups >= 1 && M % (groups * D * H * W) == 0 && stats_part != nullptr,
                "conv_gemm_group_stats: CONV3 over groups x whole samples, with a statistics buffer");
  return conv_gemm_impl(a, lda, wpacked, bias, out, ldo, nullptr, 0, 0, nullptr, mode, M, Ncols, Cpad, KG, cpg_shift,
                        D, H, W, 1, stats_part, cin_real, dtype, stream, groups, w_gstride, b_gstride);
}

// mmseg_conv_gemm_ex over `groups` equal sample groups of A / out with their own packed weights (group gi:
// wpacked + gi * w_gstride elements) and bias (bias + gi * b_gstride): the modality encoders' small levels as one
// launch (+ one split-K reduce).  Runtime-brick CONV3 shapes only (small volumes).
int mmseg_conv_gemm_group(const void* a, int lda, const void* wpacked, const float* bias, void* out, int ldo,
                          float* splitk_ws, int mode, int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H,
                          int W, int ksplit, int cin_real, int groups, long long w_gstride, int b_gstride, int dtype,
                          void* stream) {
  MMSEG_REQUIRE(mode == MODE_CONV3 && groups >= 1 && M % (groups * D * H * W) == 0,
                "conv_gemm_group: CONV3 over groups x whole samples");
  return conv_gemm_impl(a, lda, wpacked, bias, out, ldo, nullptr, 0, 0, splitk_ws, mode, M, Ncols, Cpad, KG, cpg_shift,
                        D, H, W, ksplit, nullptr, cin_real, dtype, stream, groups, w_gstride, b_gstride);
}

int mmseg_conv_gemm_ex(const void* a, int lda, const void* wpacked, const float* bias, void* out, int ldo,
                       float* splitk_ws, int mode, int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H,
                       int W, int ksplit, float* stats_part, int cin_real, int dtype, void* stream) {
  return conv_gemm_impl(a, lda, wpacked, bias, out, ldo, nullptr, 0, 0, splitk_ws, mode, M, Ncols, Cpad, KG,
                        cpg_shift, D, H, W, ksplit, stats_part, cin_real, dtype, stream);
}

// mmseg_conv_gemm_ex (no statistics) with the whole-row output hint: columns [Ncols, zcols) of the output rows are
// written as zeros by the kernels that support it (the brick2 conv kernels), left alone by the others.
int mmseg_conv_gemm_zw(const void* a, int lda, const void* wpacked, const float* bias, void* out, int ldo,
                       float* splitk_ws, int mode, int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H,
                       int W, int ksplit, int cin_real, int zcols, int dtype, void* stream) {
  return conv_gemm_impl(a, lda, wpacked, bias, out, ldo, nullptr, 0, 0, splitk_ws, mode, M, Ncols, Cpad, KG,
                        cpg_shift, D, H, W, ksplit, nullptr, cin_real, dtype, stream, 1, 0, 0, nullptr, 0, zcols);
}

// 1x1 GEMM (MODE_POINT, ksplit 1) with the MLP's GELU in its epilogue: epi 1, out = h = A W^T + bias and gelu_out
// = gelu(h) (linear1 + GELU); epi 2, out = (A W^T) * gelu'(h) with h = gelu_in (linear2's data gradient through the
// GELU) -- bitwise the GEMM followed by mmseg_gelu_fwd / mmseg_gelu_bwd.  out, gelu_in / gelu_out at pitch ldo.
int mmseg_conv_gemm_gelu(const void* a, int lda, const void* wpacked, const float* bias, void* out, int ldo,
                         const void* gelu_in, void* gelu_out, int epi, int M, int Ncols, int Cpad, int KG, int dtype,
                         void* stream) {
  MMSEG_REQUIRE((epi == 1 && gelu_out && !gelu_in) || (epi == 2 && gelu_in && !gelu_out),
                "conv_gemm_gelu: epi 1 (forward, gelu_out) or 2 (backward, gelu_in)");
  MMSEG_REQUIRE(ldo % 8 == 0 && Ncols % 8 == 0 &&
                    ((reinterpret_cast<uintptr_t>(out) | reinterpret_cast<uintptr_t>(gelu_in) |
                      reinterpret_cast<uintptr_t>(gelu_out)) & 15) == 0,
                "conv_gemm_gelu: ldo, Ncols multiples of 8, 16-B aligned buffers");
  const int KGp = (KG + 3) & ~3;
  GemmArgs g{a, lda, wpacked, bias, out, ldo, nullptr, M, Ncols, Cpad, KG, 0, 1, 1, 1, 1, KGp,
             1 /* XCD-aware block remap */, nullptr, 0, nullptr, nullptr};
  MMSEG_REQUIRE(lda % 8 == 0, "conv_gemm_gelu: lda must be a multiple of 8");
  MMSEG_REQUIRE(Cpad >= ((Ncols + (Ncols >= 64 ? 63 : 31)) / (Ncols >= 64 ? 64 : 32)) * (Ncols >= 64 ? 64 : 32),
                "conv_gemm_gelu: packed weights must be padded to the column tile (Cpad=%d, Ncols=%d)", Cpad, Ncols);
  g.epi = epi;
  g.aux = gelu_in;
  g.aux_out = gelu_out;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMSEG_BF16) return launch_gemm<bf16_t, MODE_POINT>(g, s);
  return launch_gemm<float, MODE_POINT>(g, s);
}

// 1x1 GEMM (MODE_POINT, ksplit 1) whose epilogue adds a residual: out = round(round(A W^T + bias) + res), bitwise
// mmseg_conv_gemm into a temporary followed by mmseg_add(res, temporary, out); res may alias out.  The SwinUNETR
// residual sums (UnetResBlock input gradient dx += d(conv3 branch), the MLP residual x + fc2(.)) without a pass.
int mmseg_conv_gemm_res(const void* a, int lda, const void* wpacked, const float* bias, const void* res, int ldres,
                        void* out, int ldo, int M, int Ncols, int Cpad, int KG, int dtype, void* stream) {
  MMSEG_REQUIRE(res != nullptr, "conv_gemm_res: residual required");
  return conv_gemm_impl(a, lda, wpacked, bias, out, ldo, nullptr, 0, 0, nullptr, MODE_POINT, M, Ncols, Cpad, KG, 0, 1,
                        1, 1, 1, nullptr, 0, dtype, stream, 1, 0, 0, res, ldres);
}

// mmseg_conv_gemm_ex (no fused statistics) whose output columns [split, Ncols) go to a second tensor out2 (row
// pitch ldo2) as columns 0..: the decoder's first-conv data gradient writes d(upsampled) and d(skip) dense.
int mmseg_conv_gemm_split(const void* a, int lda, const void* wpacked, const float* bias, void* out, int ldo,
                          void* out2, int ldo2, int split, float* splitk_ws, int mode, int M, int Ncols, int Cpad,
                          int KG, int cpg_shift, int D, int H, int W, int ksplit, int cin_real, int dtype,
                          void* stream) {
  MMSEG_REQUIRE(out2 && split > 0 && split < Ncols && split % 8 == 0 && ldo2 % 8 == 0 && ldo % 8 == 0 &&
                    (reinterpret_cast<uintptr_t>(out2) & 15) == 0 && mode != MODE_CONVT_FWD,
                "conv_gemm_split: split %d must be a multiple of 8 inside (0, %d), ldo / ldo2 multiples of 8, out2 "
                "16-B aligned", split, Ncols);
  return conv_gemm_impl(a, lda, wpacked, bias, out, ldo, out2, ldo2, split, splitk_ws, mode, M, Ncols, Cpad, KG,
                        cpg_shift, D, H, W, ksplit, nullptr, cin_real, dtype, stream);
}

int conv_gemm_impl(const void* a, int lda, const void* wpacked, const float* bias, void* out, int ldo, void* out2,
                   int ldo2, int split, float* splitk_ws, int mode, int M, int Ncols, int Cpad, int KG, int cpg_shift,
                   int D, int H, int W, int ksplit, float* stats_part, int cin_real, int dtype, void* stream,
                   int groups, long long w_gstride, int b_gstride, const void* res, int ldres, int zcols) {
  MMSEG_REQUIRE(zcols == 0 || (zcols >= Ncols && zcols % 8 == 0 && zcols <= ldo && !out2 && Ncols % 8 == 0 &&
                               zcols - Ncols <= 48),
                "conv_gemm: whole-row extent zcols=%d must lie in [Ncols, min(ldo, Ncols + 48)]", zcols);
  MMSEG_REQUIRE(!res || (mode == MODE_POINT && ksplit == 1 && !out2 && ldo % 8 == 0 && ldres % 8 == 0 &&
                         Ncols % 8 == 0 && ((reinterpret_cast<uintptr_t>(out) | reinterpret_cast<uintptr_t>(res)) &
                                            15) == 0),
                "conv_gemm_res: MODE_POINT, ksplit 1, pitches and Ncols multiples of 8, 16-B aligned out / res");
  MMSEG_REQUIRE(cin_real >= 0 && cin_real <= (8 << cpg_shift), "conv_gemm: cin_real %d outside [0, %d]", cin_real,
                8 << cpg_shift);
  MMSEG_REQUIRE(!stats_part || (mode == MODE_CONV3 && ksplit == 1 &&
                                (groups > 1 ? mmseg_conv3_group_stats_bricks(M, Ncols, Cpad, KG, cpg_shift, D, H, W, lda,
                                                                             ldo, dtype)
                                            : mmseg_conv3_stats_bricks(M, Ncols, Cpad, KG, cpg_shift, D, H, W, lda, ldo,
                                                                       dtype)) > 0),
                "conv_gemm_stats: fused statistics need a brick kernel without split-K for this shape");
  MMSEG_REQUIRE(lda % 8 == 0 && ldo >= 1, "conv_gemm: lda must be a multiple of 8 (got %d)", lda);
  MMSEG_REQUIRE(Cpad >= ((Ncols + (Ncols >= 64 ? 63 : 31)) / (Ncols >= 64 ? 64 : 32)) * (Ncols >= 64 ? 64 : 32),
                "conv_gemm: packed weights must be padded to the column tile (Cpad=%d, Ncols=%d)", Cpad, Ncols);
  MMSEG_REQUIRE(ksplit >= 1, "conv_gemm: ksplit >= 1");
  MMSEG_REQUIRE(ksplit == 1 || splitk_ws != nullptr, "conv_gemm: split-K needs a workspace");
  const int KGp = (KG + 3) & ~3;
  int kps = ((ceil_div(KGp, ksplit) + 3) / 4) * 4;
  ksplit = ceil_div(KGp, kps);
  GemmArgs g{a, lda, wpacked, bias, out, ldo, splitk_ws, M, Ncols, Cpad, KG, cpg_shift, D, H, W, ksplit, kps,
             1 /* XCD-aware block remap */, stats_part,
             mode == MODE_CONV3 ? (cin_real + 31) / 32 : 0, nullptr, nullptr, out2,
             ldo2, split};
  if (groups > 1) {
    g.grp_n = M / (D * H * W) / groups;
    g.w_gstride = w_gstride;
    g.b_gstride = b_gstride;
  }
  g.res = res;
  g.ldres = ldres;
  g.zcols = zcols;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMSEG_BF16) return launch_gemm_mode<bf16_t>(g, mode, s);
  return launch_gemm_mode<float>(g, mode, s);
}

// 1 when mmseg_conv3_fwd_norm can run this shape (the brick5 kernel, the only conv forward that applies a
// deferred InstanceNorm + ReLU to its input): bf16, one 32-channel input chunk, 32 output columns, W % 16.
int mmseg_conv3_norm_ok(int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H, int W, int lda, int ldo,
                        int dtype) {
  if (dtype != MMSEG_BF16 || !knob("MMSEG_DEFER_CONV_NORM", 1)) return 0;
  GemmArgs g{};
  g.lda = lda; g.ldo = ldo; g.M = M; g.Ncols = Ncols; g.Cpad = Cpad; g.KG = KG; g.cpg_shift = cpg_shift;
  g.D = D; g.H = H; g.W = W; g.ksplit = 1;
  g.out = reinterpret_cast<void*>(static_cast<uintptr_t>(256));   // the caller's output is 16-B aligned (checked)
  return brick5_selected(g, 2) ? 1 : 0;
}

// 3^3 conv forward of an A source holding the PRE-norm activation of an InstanceNorm + ReLU: the kernel stages
// relu((a - nmean[n][c]) * nrstd[n][c]) rounded to bf16, exactly the values mmseg_instnorm_relu_fwd would
// write, so that output never has to be materialised (requires mmseg_conv3_norm_ok).
int mmseg_conv3_fwd_norm(const void* a, int lda, const float* nmean, const float* nrstd, const void* wpacked,
                         const float* bias, void* out, int ldo, int M, int Ncols, int Cpad, int KG, int cpg_shift,
                         int D, int H, int W, int dtype, void* stream) {
  MMSEG_REQUIRE(nmean && nrstd && (reinterpret_cast<uintptr_t>(out) & 15) == 0 &&
                    mmseg_conv3_norm_ok(M, Ncols, Cpad, KG, cpg_shift, D, H, W, lda, ldo, dtype),
                "conv3_fwd_norm: unsupported shape (mmseg_conv3_norm_ok)");
  const int KGp = (KG + 3) & ~3;
  GemmArgs g{a, lda, wpacked, bias, out, ldo, nullptr, M, Ncols, Cpad, KG, cpg_shift, D, H, W, 1, KGp,
             1 /* XCD-aware block remap */, nullptr, 0, nmean, nrstd};
  return launch_gemm<bf16_t, MODE_CONV3>(g, (hipStream_t)stream);
}

// Mixed bf16/fp8 forward (config c5): the brick6 shapes of a 3^3 conv with e4m3 operands and fp32 accumulation.
int mmseg_conv3_fp8_ok(int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H, int W, int lda, int ldo) {
  GemmArgs g{};
  g.lda = lda; g.ldo = ldo; g.M = M; g.Ncols = Ncols; g.Cpad = Cpad; g.KG = KG; g.cpg_shift = cpg_shift;
  g.D = D; g.H = H; g.W = W; g.ksplit = 1;
  g.out = reinterpret_cast<void*>(static_cast<uintptr_t>(256));
  return brick5_selected(g, 2) ? 1 : 0;
}

int mmseg_pack_conv3_fp8(const float* w, int Co, int Ci, int Cip, int KGp, int Cpad, void* dst, float* wdq,
                         void* stream) {
  MMSEG_REQUIRE(w && dst && wdq && Co > 0 && Co <= Cpad && Ci <= Cip && Cip % 8 == 0 && KGp * 8 >= 27 * Cip,
                "pack_conv3_fp8: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  hipMemsetAsync(dst, 0, (size_t)KGp * Cpad * 8, s);   // K / column padding stays e4m3 zero
  MMSEG_LAUNCH(pack_conv3_fp8_kernel, dim3(Co), dim3(256), 0, s, w, Ci, Cip, Cpad, (unsigned char*)dst, wdq);
  return mmseg::check_launch("pack_conv3_fp8");
}

// out = conv3(A) with e4m3 operands (A: bf16 NDHWC, staged as e4m3; with nmean / nrstd: relu((a - mean) * rstd)
// first, as mmseg_conv3_fwd_norm), bf16 output; w8 / wdq from mmseg_pack_conv3_fp8 (requires mmseg_conv3_fp8_ok).
int mmseg_conv3_fwd_fp8(const void* a, int lda, const float* nmean, const float* nrstd, const void* w8,
                        const float* wdq, const float* bias, void* out, int ldo, int M, int Ncols, int Cpad, int KG,
                        int cpg_shift, int D, int H, int W, void* stream) {
  MMSEG_REQUIRE(a && w8 && wdq && out && (nmean == nullptr) == (nrstd == nullptr) &&
                    (reinterpret_cast<uintptr_t>(out) & 15) == 0 &&
                    mmseg_conv3_fp8_ok(M, Ncols, Cpad, KG, cpg_shift, D, H, W, lda, ldo),
                "conv3_fwd_fp8: unsupported shape (mmseg_conv3_fp8_ok)");
  const int KGp = (KG + 3) & ~3;
  GemmArgs g{a, lda, w8, bias, out, ldo, nullptr, M, Ncols, Cpad, KG, cpg_shift, D, H, W, 1, KGp,
             1 /* XCD-aware block remap */, nullptr, 0, nmean, nrstd};
  g.wdq = wdq;
  launch_brick5(g, (hipStream_t)stream);
  return mmseg::check_launch("conv3_fwd_fp8");
}

// Chunks per sample of the InstanceNorm-backward partials mmseg_conv3_dgrad_in writes for this CONV3 data-gradient
// shape (the brick5 kernel's blocks per column tile), or 0 when that kernel does not run it.
int mmseg_conv3_dgrad_in_chunks(int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H, int W, int lda,
                                int ldo, int dtype) {
  if (dtype != MMSEG_BF16) return 0;
  GemmArgs g{};
  g.lda = lda; g.ldo = ldo; g.M = M; g.Ncols = Ncols; g.Cpad = Cpad; g.KG = KG; g.cpg_shift = cpg_shift;
  g.D = D; g.H = H; g.W = W; g.ksplit = 1;
  g.out = reinterpret_cast<void*>(static_cast<uintptr_t>(256));   // the caller's output is 16-B aligned (checked)
  if (!brick5_selected(g, 2)) return 0;
  const int nt_n = Ncols / 32;
  const int per_nt = std::max(1, knob("MMSEG_BRICK4_BLOCKS", 256) / nt_n);
  const int nb5 = (M / (D * H * W)) * (D / 4) * (H / 4) * (W / 16);
  const int upb5 = ceil_div(nb5, std::min(per_nt, nb5));
  return ceil_div(nb5, upb5);
}

// CONV3 data gradient (mmseg_conv_gemm_ex, ksplit 1, no bias) whose output dy feeds the backward of an InstanceNorm +
// ReLU with pre-norm input inx (pitch ldinx) and statistics inmean / inrstd [N][Ncols]: the kernel also writes that
// backward's partial sums inpart [N][mmseg_conv3_dgrad_in_chunks()][Ncols][2] (the layout mmseg_instnorm_bwd_part
// reads), so its partial pass over x and dy is skipped.
int mmseg_conv3_dgrad_in(const void* a, int lda, const void* wpacked, void* out, int ldo, int M, int Ncols, int Cpad,
                         int KG, int cpg_shift, int D, int H, int W, const void* inx, int ldinx, const float* inmean,
                         const float* inrstd, float* inpart, int dtype, void* stream) {
  MMSEG_REQUIRE(inx && inmean && inrstd && inpart && ldinx % 8 == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0 &&
                    mmseg_conv3_dgrad_in_chunks(M, Ncols, Cpad, KG, cpg_shift, D, H, W, lda, ldo, dtype) > 0,
                "conv3_dgrad_in: unsupported shape (mmseg_conv3_dgrad_in_chunks)");
  const int KGp = (KG + 3) & ~3;
  GemmArgs g{a, lda, wpacked, nullptr, out, ldo, nullptr, M, Ncols, Cpad, KG, cpg_shift, D, H, W, 1, KGp,
             1 /* XCD-aware block remap */, nullptr, 0, nullptr, nullptr};
  g.inx = inx;
  g.ldinx = ldinx;
  g.inmean = inmean;
  g.inrstd = inrstd;
  g.inpart = inpart;
  launch_brick5(g, (hipStream_t)stream);
  return mmseg::check_launch("conv3_dgrad_in");
}

// Number of K splits the CONV3 path wants for this shape (callers size the
// split-K workspace, ksplit*M*Ncols floats, with it and pass it as ksplit).
// 1 when mmseg_conv_gemm_group / mmseg_conv3_wgrad_group take this shape: the runtime-brick conv (plan kind 2)
// and, for the weight gradient, the runtime-brick weight-gradient kernel (kind 3).
// (a grouped launch takes the runtime-brick kernels; MMSEG_GROUP_FORCE_R (default on) also groups shapes that would
// otherwise take the (4, 8, 8)-brick family -- the 24^3 / 48^3 levels: one launch over both modalities on the
// runtime-brick kernels beat two on the brick family there, r04j / r04l / r04n A/B -0.05..-0.07 ms per step)
int mmseg_conv3_group_ok(int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H, int W, int lda, int ldo,
                         int dtype) {
  if (!knob("MMSEG_GROUP_SMALL", 1)) return 0;
  const int ts = dtype == MMSEG_BF16 ? 2 : 4;
  if (plan_conv3(M, Ncols, 8 << cpg_shift, D, H, W, lda, ldo, ts).kind == 2) return 1;
  return knob("MMSEG_GROUP_FORCE_R", 1) && plan_conv3(M, Ncols, 8 << cpg_shift, D, H, W, lda, ldo, ts, true).kind == 2
             ? 1 : 0;
}
int mmseg_conv3_wgrad_group_ok(long long V, int Co, int Cip, int Ci, int cpg_shift, int D, int H, int W, int lddy,
                               int ldx, int dtype) {
  if (!knob("MMSEG_GROUP_SMALL", 1)) return 0;
  if (plan_conv3_wgrad(V, Co, Cip, Ci, cpg_shift, D, H, W, lddy, ldx, dtype, 1LL << 40).kind == 3) return 1;
  return knob("MMSEG_GROUP_FORCE_R", 1) &&
                 plan_conv3_wgrad(V, Co, Cip, Ci, cpg_shift, D, H, W, lddy, ldx, dtype, 1LL << 40, true).kind == 3
             ? 1 : 0;
}
// split count of a grouped conv (mmseg_conv_gemm_group): the runtime-brick plan's
// Bricks per sample for which the grouped (forced runtime-brick) conv can emit fused InstanceNorm partials
// (mmseg_conv_gemm_group_stats): none (see the function).
int mmseg_conv3_group_stats_bricks(int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H, int W, int lda,
                                   int ldo, int dtype) {
  return 0;   // (as mmseg_conv3_stats_bricks: equal per step, r04ad -- the epilogue costs what the pass did)
}

int mmseg_conv3_group_splits(int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H, int W, int lda, int ldo,
                             int dtype) {
  const Conv3Plan p = plan_conv3(M, Ncols, 8 << cpg_shift, D, H, W, lda, ldo, dtype == MMSEG_BF16 ? 2 : 4, true);
  return p.kind == 2 ? p.ks : 1;
}

int mmseg_conv3_splits(int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H, int W, int lda, int ldo,
                       int dtype) {
  const int tsize = dtype == MMSEG_BF16 ? 2 : 4;
  const Conv3Plan p = plan_conv3(M, Ncols, 8 << cpg_shift, D, H, W, lda, ldo, tsize);
  if (p.kind == 2) return p.ks;
  if (p.kind == 1) return 1;
  // per-lane gather GEMM: enough (128 x 64|32) tiles to fill the chip
  const int tiles = ceil_div(M, 128) * ceil_div(Ncols, Ncols >= 64 ? 64 : 32);
  if (tiles >= 512 || KG < 32) return 1;
  int ks = ceil_div(512, tiles);
  if (ks > KG / 16) ks = KG / 16;
  return ks < 1 ? 1 : ks;
}

// Weight-gradient partials: part[ksplit][Ca][Ncols] (fp32).
int mmseg_wgrad(const void* a, int lda, const void* b, int ldb, float* part, float* bias_part, int mode, int Ca,
                int Ncols, int cpg_shift, long long V, int D, int H, int W, int ksplit, int dtype, void* stream) {
  MMSEG_REQUIRE(Ca % 8 == 0, "wgrad: rows (%d) must be a multiple of 8", Ca);
  MMSEG_REQUIRE(Ncols % 8 == 0, "wgrad: cols (%d) must be a multiple of 8", Ncols);
  MMSEG_REQUIRE(V < (1LL << 31), "wgrad: voxel count %lld must fit 31 bits", V);
  // legacy entry (tap-major partials + mmseg_wgrad_reduce): brick kinds 2/3 write channel-major tiles and
  // are reached through mmseg_conv3_wgrad only
  int brick = mode == MODE_CONV3 ? wgrad_brick_ok(Ca, cpg_shift, D, H, W, lda, ldb, dtype) : 0;
  if (brick > 1) brick = 1;
  long long vps = ((V + ksplit - 1) / ksplit + 63) / 64 * 64;
  if (brick) {
    ksplit = brick_wgrad_splits(V, ksplit, Ca, cpg_shift, brick, D, H, W);
  } else {
    ksplit = (int)((V + vps - 1) / vps);
  }
  WgradArgs g{a, lda, b, ldb, part, bias_part, Ca, Ncols, cpg_shift, V, D, H, W, ksplit, vps,
              1, brick, nullptr, nullptr, 0};
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMSEG_BF16) {
    switch (mode) {
      case MODE_CONV3: return launch_wgrad<bf16_t, MODE_CONV3>(g, s);
      case MODE_POINT: return launch_wgrad<bf16_t, MODE_POINT>(g, s);
      case MODE_CONVT_DGRAD: return launch_wgrad<bf16_t, MODE_CONVT_DGRAD>(g, s);
    }
  } else {
    switch (mode) {
      case MODE_CONV3: return launch_wgrad<float, MODE_CONV3>(g, s);
      case MODE_POINT: return launch_wgrad<float, MODE_POINT>(g, s);
      case MODE_CONVT_DGRAD: return launch_wgrad<float, MODE_CONVT_DGRAD>(g, s);
    }
  }
  mmseg::set_error("wgrad: bad mode %d", mode);
  return 1;
}

// Effective split count the wgrad launcher will use (callers size `part` with it).
int mmseg_wgrad_splits(long long V, int ksplit) { return mmseg_wgrad_splits_impl(V, ksplit); }

// Same for the CONV3 brick path (splits the list of 4x4x8 bricks).
int mmseg_wgrad_splits_conv3(long long V, int ksplit, int Ca, int cpg_shift, int D, int H, int W, int lda, int ldb,
                             int dtype) {
  int kind = wgrad_brick_ok(Ca, cpg_shift, D, H, W, lda, ldb, dtype);
  if (kind > 1) kind = 1;   // the legacy entry's kernels (see mmseg_wgrad)
  if (!kind) return mmseg_wgrad_splits(V, ksplit);
  return brick_wgrad_splits(V, ksplit, Ca, cpg_shift, kind, D, H, W);
}

int mmseg_wgrad_reduce(const float* part, float* grad, const float* bias_part, float* bias_grad, int Ca, int Ncols,
                       int ksplit, int cpad, int creal, int ntap, int accumulate, void* stream) {
  MMSEG_REQUIRE(((long long)Ca * Ncols) % 4 == 0 && (reinterpret_cast<uintptr_t>(part) & 15) == 0,
                "wgrad_reduce: Ca*Ncols %% 4 == 0 and a 16-B aligned partial buffer");
  WReduceArgs g{part, grad, bias_part, bias_grad, Ca, Ncols, ksplit, cpad, creal, ntap, accumulate, 0};
  return launch_wgrad_reduce(g, stream);
}

// mmseg_wgrad_reduce queued until mmseg_wgrad_reduce_flush(stream) (part must stay untouched until then)
int mmseg_wgrad_reduce_defer(const float* part, float* grad, const float* bias_part, float* bias_grad, int Ca,
                             int Ncols, int ksplit, int cpad, int creal, int ntap, int accumulate, void* stream) {
  MMSEG_REQUIRE(((long long)Ca * Ncols) % 4 == 0 && (reinterpret_cast<uintptr_t>(part) & 15) == 0,
                "wgrad_reduce: Ca*Ncols %% 4 == 0 and a 16-B aligned partial buffer");
  WReduceArgs g{part, grad, bias_part, bias_grad, Ca, Ncols, ksplit, cpad, creal, ntap, accumulate, 0};
  return wred_push(g, 1, stream);
}

// Weight (+ bias) gradient of a 3^3 conv straight into the torch-layout fp32 gradient
// grad[Co][Ci][27] (+ bias_grad[Co]), = or += (accumulate).  The library picks kernel and split;
// ws holds mmseg_conv3_wgrad_ws_floats() floats (more lets it split further, fewer is clamped).
long long mmseg_conv3_wgrad_ws_floats(long long V, int Co, int Cip, int Ci, int cpg_shift, int D, int H, int W,
                                      int lddy, int ldx, int dtype) {
  const long long cap = 16LL << 20;
  return plan_conv3_wgrad(V, Co, Cip, Ci, cpg_shift, D, H, W, lddy, ldx, dtype, cap).ws;
}

// Grouped weight gradient (mmseg_conv3_wgrad_group): the plan of the whole V, its split count rounded down to a
// multiple of `groups` (at least one split per group), never direct.
Conv3WgradPlan plan_conv3_wgrad_grouped(long long V, int Co, int Cip, int Ci, int cpg_shift, int D, int H, int W,
                                        int lda, int ldb, int dtype, long long ws_cap, int groups) {
  Conv3WgradPlan p = plan_conv3_wgrad(V, Co, Cip, Ci, cpg_shift, D, H, W, lda, ldb, dtype, ws_cap, groups > 1);
  if (groups <= 1) return p;
  p.ksplit = p.ksplit / groups * groups;
  if (p.ksplit < groups) p.ksplit = groups;
  // one split per group (the deepest levels): each writes its group's gradient directly, as the ungrouped
  // single-split launch does -- a reduce would only copy 2 x 28 MB there (28.8 us, r04d)
  p.direct = p.kind >= 2 && p.ksplit == groups && Ci == Cip;
  p.ws = p.direct ? 0 : (long long)p.ksplit * ((long long)Co * 27 * Cip + Co);
  return p;
}

long long mmseg_conv3_wgrad_group_ws_floats(long long V, int Co, int Cip, int Ci, int cpg_shift, int D, int H, int W,
                                            int lddy, int ldx, int groups, int dtype) {
  const long long cap = 16LL << 20;
  return plan_conv3_wgrad_grouped(V, Co, Cip, Ci, cpg_shift, D, H, W, lddy, ldx, dtype, cap, groups).ws;
}

int conv3_wgrad_impl(const void* dy, int lddy, const void* x, int ldx, const float* nmean, const float* nrstd,
                     float* grad, float* bias_grad, int Co, int Cip, int Ci, int cpg_shift, long long V, int D, int H,
                     int W, float* ws, long long ws_floats, int accumulate, int dtype, void* stream, int phase = 3,
                     int groups = 1, long long grad_gstride = 0, int bias_gstride = 0);

// The weight / bias gradients of `groups` same-shape 3^3 convs over equal sample groups of one activation pair
// (group gi: samples [gi N / groups, (gi + 1) N / groups) of dy / x, gradient at grad + gi * grad_gstride and
// bias_grad + gi * bias_gstride floats) in one weight-gradient launch and one reduce -- the modality encoders'
// small levels.  Runtime-brick weight-gradient shapes only; ws: mmseg_conv3_wgrad_group_ws_floats().
int mmseg_conv3_wgrad_group(const void* dy, int lddy, const void* x, int ldx, float* grad, float* bias_grad, int Co,
                            int Cip, int Ci, int cpg_shift, long long V, int D, int H, int W, float* ws,
                            long long ws_floats, int accumulate, int groups, long long grad_gstride,
                            int bias_gstride, int phase, int dtype, void* stream) {
  MMSEG_REQUIRE(groups >= 1 && V % ((long long)groups * D * H * W) == 0 && phase >= 1 && phase <= 7 && (phase & 3),
                "conv3_wgrad_group: V must hold groups x whole samples, phase bits 1 | 2 (| 4 defer)");
  return conv3_wgrad_impl(dy, lddy, x, ldx, nullptr, nullptr, grad, bias_grad, Co, Cip, Ci, cpg_shift, V, D, H, W, ws,
                          ws_floats, accumulate, dtype, stream, phase, groups, grad_gstride, bias_gstride);
}

int mmseg_conv3_wgrad(const void* dy, int lddy, const void* x, int ldx, float* grad, float* bias_grad, int Co, int Cip,
                      int Ci, int cpg_shift, long long V, int D, int H, int W, float* ws, long long ws_floats,
                      int accumulate, int dtype, void* stream) {
  return conv3_wgrad_impl(dy, lddy, x, ldx, nullptr, nullptr, grad, bias_grad, Co, Cip, Ci, cpg_shift, V, D, H, W, ws,
                          ws_floats, accumulate, dtype, stream);
}

// 1 when mmseg_conv3_wgrad_norm can run this shape: the brick2 weight-gradient kernel (the only one that applies
// a deferred InstanceNorm + ReLU to x), no channel padding, bf16.
int mmseg_conv3_wgrad_norm_ok(long long V, int Co, int Cip, int Ci, int cpg_shift, int D, int H, int W, int lddy,
                              int ldx, int dtype) {
  if (dtype != MMSEG_BF16 || Ci != Cip || !knob("MMSEG_DEFER_CONV_NORM", 1)) return 0;
  return plan_conv3_wgrad(V, Co, Cip, Ci, cpg_shift, D, H, W, lddy, ldx, dtype, 1LL << 40).kind == 2 ? 1 : 0;
}

// mmseg_conv3_wgrad with x the PRE-norm activation of an InstanceNorm + ReLU ([N][Cip] mean / rstd), applied on
// staging exactly as mmseg_instnorm_relu_fwd would write it (requires mmseg_conv3_wgrad_norm_ok).
int mmseg_conv3_wgrad_norm(const void* dy, int lddy, const void* x, int ldx, const float* nmean, const float* nrstd,
                           float* grad, float* bias_grad, int Co, int Cip, int Ci, int cpg_shift, long long V, int D,
                           int H, int W, float* ws, long long ws_floats, int accumulate, int dtype, void* stream) {
  MMSEG_REQUIRE(nmean && nrstd && mmseg_conv3_wgrad_norm_ok(V, Co, Cip, Ci, cpg_shift, D, H, W, lddy, ldx, dtype),
                "conv3_wgrad_norm: unsupported shape (mmseg_conv3_wgrad_norm_ok)");
  return conv3_wgrad_impl(dy, lddy, x, ldx, nmean, nrstd, grad, bias_grad, Co, Cip, Ci, cpg_shift, V, D, H, W, ws,
                          ws_floats, accumulate, dtype, stream);
}

// mmseg_conv3_wgrad in two phases (bit 1: the weight-gradient kernel, bit 2: the split reduce), so a caller can
// time the kernel alone; nmean / nrstd optional (deferred norm of x, see mmseg_conv3_wgrad_norm).
int mmseg_conv3_wgrad_ex(const void* dy, int lddy, const void* x, int ldx, const float* nmean, const float* nrstd,
                         float* grad, float* bias_grad, int Co, int Cip, int Ci, int cpg_shift, long long V, int D,
                         int H, int W, float* ws, long long ws_floats, int accumulate, int phase, int dtype,
                         void* stream) {
  MMSEG_REQUIRE(phase >= 1 && phase <= 15 && (phase & 3) && (!(phase & 8) || (Co >= 16 && Co % 16 == 0)),
                "conv3_wgrad_ex: phase %d: bits 1 | 2 (| 4 defer, | 8 last 16 rows padding)", phase);
  MMSEG_REQUIRE(!nmean || (nrstd && mmseg_conv3_wgrad_norm_ok(V, Co, Cip, Ci, cpg_shift, D, H, W, lddy, ldx, dtype)),
                "conv3_wgrad_ex: unsupported shape for the deferred norm (mmseg_conv3_wgrad_norm_ok)");
  return conv3_wgrad_impl(dy, lddy, x, ldx, nmean, nrstd, grad, bias_grad, Co, Cip, Ci, cpg_shift, V, D, H, W, ws,
                          ws_floats, accumulate, dtype, stream, phase);
}

// Launch the reduces deferred with phase bit 4 (in the order they were deferred, at most WRB_MAX per launch) on
// `stream`; each gradient is bitwise what its own reduce would have written.  Returns the number flushed.
int mmseg_wgrad_reduce_flush(void* stream) {
  int done = 0;
  std::vector<PendingWred> keep;
  std::vector<PendingWred> mine;
  for (auto& e : g_wred_pending) (e.stream == stream ? mine : keep).push_back(e);
  g_wred_pending.swap(keep);
  for (size_t i0 = 0; i0 < mine.size(); i0 += 0) {
    WReduceBatch b{};
    // at most WRB_MAX per launch, and a gradient written by two queued reduces (an accumulating second use) starts
    // a new launch, so the two stay ordered
    size_t i1 = i0;
    while (i1 < mine.size() && i1 - i0 < (size_t)WRB_MAX) {
      bool clash = false;
      for (size_t j = i0; j < i1; ++j)
        clash = clash || mine[j].r.grad == mine[i1].r.grad ||
                (mine[i1].r.bias_grad != nullptr && mine[j].r.bias_grad == mine[i1].r.bias_grad);
      if (clash) break;
      ++i1;
    }
    b.n = (int)(i1 - i0);
    int blk = 0;
    for (int k = 0; k < b.n; ++k) {
      const PendingWred& e = mine[i0 + k];
      const long long total = (long long)e.r.Ca * e.r.Ncols + (e.r.bias_part ? e.r.Ca : 0);
      b.d[k] = e.r;
      b.S[k] = wred_slices(e.r);
      b.nbx[k] = ceil_div(total, 1024 / b.S[k]);
      b.blk0[k] = blk;
      blk += b.nbx[k] * e.groups;
    }
    b.blk0[b.n] = blk;
    mmseg::note_kernel("wgrad_reduce_batch_kernel");
    MMSEG_LAUNCH(wgrad_reduce_batch_kernel, dim3(blk), dim3(256), 0, (hipStream_t)stream, b);
    if (mmseg::check_launch("wgrad_reduce_batch")) return -1;
    done += b.n;
    i0 = i1;
  }
  return done;
}

// number of deferred reduces not yet flushed (all streams)
int mmseg_wgrad_reduce_pending(void) { return (int)g_wred_pending.size(); }

// drop the deferred reduces of `stream` (a backward that failed half way); returns how many
int mmseg_wgrad_reduce_discard(void* stream) {
  const size_t n0 = g_wred_pending.size();
  g_wred_pending.erase(std::remove_if(g_wred_pending.begin(), g_wred_pending.end(),
                                      [&](const PendingWred& e) { return e.stream == stream; }),
                       g_wred_pending.end());
  return (int)(n0 - g_wred_pending.size());
}

int conv3_wgrad_impl(const void* dy, int lddy, const void* x, int ldx, const float* nmean, const float* nrstd,
                     float* grad, float* bias_grad, int Co, int Cip, int Ci, int cpg_shift, long long V, int D, int H,
                     int W, float* ws, long long ws_floats, int accumulate, int dtype, void* stream, int phase,
                     int groups, long long grad_gstride, int bias_gstride) {
  MMSEG_REQUIRE(Co % 8 == 0 && Cip % 8 == 0 && Ci <= Cip && (8 << cpg_shift) == Cip,
                "conv3_wgrad: Co=%d, Cip=%d must be multiples of 8, Ci=%d <= Cip, Cip = 8 << cpg_shift", Co, Cip, Ci);
  const Conv3WgradPlan p = plan_conv3_wgrad_grouped(V, Co, Cip, Ci, cpg_shift, D, H, W, lddy, ldx, dtype, ws_floats,
                                                    groups);
  MMSEG_REQUIRE(!nmean || p.kind == 2, "conv3_wgrad: a deferred norm needs the brick2 weight-gradient kernel");
  MMSEG_REQUIRE(groups <= 1 || p.kind == 3, "conv3_wgrad_group: only the runtime-brick weight gradient is grouped");
  MMSEG_REQUIRE(p.ws <= ws_floats && (p.ws == 0 || ws != nullptr), "conv3_wgrad: workspace of %lld floats < %lld",
                ws_floats, p.ws);
  const int ncols = 27 * Cip;
  float* part = p.direct ? nullptr : ws;
  float* bpart = (p.direct || bias_grad == nullptr) ? nullptr : ws + (long long)p.ksplit * Co * ncols;
  const long long vps = ((V + p.ksplit - 1) / p.ksplit + 63) / 64 * 64;
  // XCD swizzle: each XCD walks a contiguous range of (split, row tile, channel chunk) tiles,
  // so the chunks of one brick range -- which all read the same dy -- and neighbouring brick ranges -- which share
  // halo planes -- meet in one L2 (r04e A/B: 6.38 -> 6.35 ms/step)
  WgradArgs g{dy, lddy, x, ldx, part, p.direct ? bias_grad : bpart, Co, ncols, cpg_shift, V, D, H, W, p.ksplit, vps,
              1, p.kind, p.direct ? grad : nullptr, p.direct ? bias_grad : nullptr,
              accumulate, wgrad_kchunks(Cip, Ci), nmean, nrstd};
  hipStream_t s = (hipStream_t)stream;
  g.groups = groups > 1 ? groups : 0;
  g.pad16 = (phase & 8) ? 1 : 0;
  // the row-slab kernel writes fragment-native partials only (2 co tiles of 16)
  const int fmt = wgrad_row_ok(g, dtype == MMSEG_BF16 ? 2 : 4) ? 2
                  : wgrad_dma_mt(g, dtype == MMSEG_BF16 ? 2 : 4);
  g.frag = fmt > 0;
  g.groups = groups > 1 ? groups : 0;
  g.grad_gstride = grad_gstride;
  g.bias_gstride = bias_gstride;
  g.pad16 = (phase & 8) ? 1 : 0;
  g.grad_ld = p.direct ? 27 * Ci : 0;
  if (phase & 1) {
    const int rc = dtype == MMSEG_BF16 ? launch_wgrad<bf16_t, MODE_CONV3>(g, s) : launch_wgrad<float, MODE_CONV3>(g, s);
    if (rc) return rc;
  }
  if (p.direct || !(phase & 2)) return 0;
  const int ng = groups > 1 ? groups : 1;
  WReduceArgs r{part, grad, bpart, bias_grad, Co, ncols, p.ksplit / ng, Cip, Ci, 27, accumulate, p.kind >= 2 ? 1 : 0,
                fmt, wgrad_nchunk(cpg_shift, g.kchunks), grad_gstride, bias_gstride};
  r.vec4 = r.chmajor && !r.frag_mt && ((uintptr_t)grad & 15) == 0 &&
           (ng == 1 || grad_gstride % 4 == 0) && r.Ncols % 4 == 0 && ((long long)r.creal * r.ntap) % 4 == 0;
  if (phase & 4) {   // deferred: summed by the next mmseg_wgrad_reduce_flush on this stream
    return wred_push(r, ng, stream);
  }
  return launch_wgrad_reduce(r, stream, ng);
}

// Bias gradient: out[c] (+)= sum_v dy[v][c]; part must hold nblk*C floats.
int mmseg_colsum(const void* dy, int ld, int C, long long V, float* part, int nblk, float* out, int accumulate,
                 int dtype, void* stream) {
  MMSEG_REQUIRE(C % 8 == 0 && C / 8 <= 256, "colsum: C=%d must be a multiple of 8 and <= 2048", C);
  long long vps = (V + nblk - 1) / nblk;
  nblk = (int)((V + vps - 1) / vps);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMSEG_BF16)
    MMSEG_LAUNCH(colsum_partial_kernel<bf16_t>, dim3(nblk), dim3(256), 0, s, (const bf16_t*)dy, ld, C, V, vps,
                       part);
  else
    MMSEG_LAUNCH(colsum_partial_kernel<float>, dim3(nblk), dim3(256), 0, s, (const float*)dy, ld, C, V, vps,
                       part);
  if (mmseg::check_launch("colsum_partial")) return 1;
  MMSEG_LAUNCH(colsum_reduce_kernel, dim3(C), dim3(256), 0, s, part, nblk, C, out, accumulate);
  return mmseg::check_launch("colsum_reduce");
}

// out[c] (=, or += with accumulate) = sum over b < nblk of part[b][c], fixed order; the transposed conv's bias
// gradient from mmseg_wgrad's CONVT column-sum partials is mmseg_colsum_reduce(bias_part, 8 * ksplit, Cout, ...).
int mmseg_colsum_reduce(const float* part, int nblk, int C, float* out, int accumulate, void* stream) {
  MMSEG_REQUIRE(nblk >= 1 && C >= 1, "colsum_reduce: nblk, C >= 1");
  MMSEG_LAUNCH(colsum_reduce_kernel, dim3(C), dim3(256), 0, (hipStream_t)stream, part, nblk, C, out,
                     accumulate);
  return mmseg::check_launch("colsum_reduce");
}

}  // extern "C"
