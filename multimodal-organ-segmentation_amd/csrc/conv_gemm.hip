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

namespace {

enum GatherMode { MODE_CONV3 = 0, MODE_POINT = 1, MODE_CONVT_FWD = 2, MODE_CONVT_DGRAD = 3 };

struct GemmArgs {
  const void* a;  int lda;   // A source (NDHWC)
  const void* b;             // packed weights [KGp][Cpad][8]
  const float* bias;         // per output channel, or null
  void* out;      int ldo;   // output (NDHWC) for ksplit == 1
  float* part;               // [ksplit][M][Ncols] fp32 partials for ksplit > 1
  int M, Ncols, Cpad, KG, cpg_shift;
  int D, H, W;               // row grid
  int ksplit, kg_per_split;  // k-groups per split (multiple of 4)
};

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
  if (MODE == MODE_CONV3) {
    int x = (int)(m % g.W);
    long long t = m / g.W;
    int y = (int)(t % g.H);
    t /= g.H;
    int z = (int)(t % g.D);
    r.tmask = tap_valid_mask(z, y, x, g.D, g.H, g.W);
  } else if (MODE == MODE_CONVT_DGRAD) {
    int x = (int)(m % g.W);
    long long t = m / g.W;
    int y = (int)(t % g.H);
    t /= g.H;
    int z = (int)(t % g.D);
    long long n = t / g.D;
    long long H2 = 2LL * g.H, W2 = 2LL * g.W, D2 = 2LL * g.D;
    r.base = ((n * D2 + 2 * z) * H2 + 2 * y) * W2 + 2 * x;
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
  } else {
    int a = t >> 2, b = (t >> 1) & 1, c = t & 1;
    return ((long long)a * (2LL * g.H) + b) * (2LL * g.W) + c;
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

// Block = WM x WN waves; wave tile = (RM*16) x (RN*16).
template <typename T, int MODE, int WM, int WN, int RM, int RN>
__global__ __launch_bounds__(256) void conv_gemm_kernel(GemmArgs g) {
  constexpr int BM = WM * RM * 16;
  constexpr int BN = WN * RN * 16;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const long long m0 = (long long)blockIdx.x * BM + wm * RM * 16;
  const int n0 = blockIdx.y * BN + wn * RN * 16;
  const int ks = blockIdx.z;
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
#pragma unroll
  for (int i = 0; i < RM; ++i) {
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      const int col = n0 + j * 16 + (lane & 15);
      if (col >= g.Ncols) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long long row = m0 + i * 16 + (lane >> 4) * 4 + r;
        if (row >= g.M) continue;
        float v = acc[i][j][r];
        if (g.ksplit > 1) {
          g.part[((long long)ks * g.M + row) * g.Ncols + col] = v;
          continue;
        }
        if (MODE == MODE_CONVT_FWD) {
          const int t = col / Cout, co = col - t * Cout;
          if (g.bias) v += g.bias[co];
          // child voxel of input voxel `row` for tap t
          const int x = (int)(row % g.W);
          long long q = row / g.W;
          const int y = (int)(q % g.H);
          q /= g.H;
          const int z = (int)(q % g.D);
          const long long n = q / g.D;
          const long long child = ((n * 2LL * g.D + 2 * z + (t >> 2)) * 2LL * g.H + 2 * y + ((t >> 1) & 1)) * 2LL * g.W +
                                  2 * x + (t & 1);
          O[child * g.ldo + co] = from_f<T>(v);
        } else {
          if (g.bias) v += g.bias[col];
          O[row * g.ldo + col] = from_f<T>(v);
        }
      }
    }
  }
}

// Fixed-order split-K reduction for the forward GEMM: out = sum_k part[k] (+bias).
template <typename T, int MODE>
__global__ void gemm_splitk_reduce(GemmArgs g) {
  long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  long long total = (long long)g.M * g.Ncols;
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
    const int x = (int)(row % g.W);
    long long q = row / g.W;
    const int y = (int)(q % g.H);
    q /= g.H;
    const int z = (int)(q % g.D);
    const long long n = q / g.D;
    const long long child = ((n * 2LL * g.D + 2 * z + (t >> 2)) * 2LL * g.H + 2 * y + ((t >> 1) & 1)) * 2LL * g.W +
                            2 * x + (t & 1);
    O[child * g.ldo + co] = from_f<T>(v);
  } else {
    if (g.bias) v += g.bias[col];
    O[row * g.ldo + col] = from_f<T>(v);
  }
}

// ------------------------------------------------------------------ wgrad
// part[ks][row][col] = sum_{v in split ks} A[v][row] * Bgather[v][col]
//   CONV3 : A = dy (rows = Cout), B = x at v + off(tap), col = tap*Cin + ci
//   POINT : A = dy, B = x at v
//   CONVT : A = x (rows = Cin), B = dy at child(v, tap), col = tap*Cout + co
struct WgradArgs {
  const void* a;  int lda;
  const void* b;  int ldb;
  float* part;
  int Ca, Ncols, cpg_shift;
  long long V;               // voxels in the a-grid
  int D, H, W;
  int ksplit;
  long long vox_per_split;   // multiple of KV
};

template <typename T, int MODE, int WM, int WN, int RM, int RN, int KV>
__global__ __launch_bounds__(256) void wgrad_kernel(WgradArgs g) {
  constexpr int BM = WM * RM * 16;
  constexpr int BN = WN * RN * 16;
  constexpr int PAD = 16 / sizeof(T);
  constexpr int LDS_ROW = KV + PAD;   // elements
  __shared__ __attribute__((aligned(16))) T As[BM * LDS_ROW];
  __shared__ __attribute__((aligned(16))) T Bs[BN * LDS_ROW];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int row0 = blockIdx.y * BM;
  const int col0 = blockIdx.x * BN;
  const int ks = blockIdx.z;
  const long long v_begin = ks * g.vox_per_split;
  long long v_end = v_begin + g.vox_per_split;
  if (v_end > g.V) v_end = g.V;

  const T* A = reinterpret_cast<const T*>(g.a);
  const T* B = reinterpret_cast<const T*>(g.b);

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  constexpr int AG = BM / 8;  // 8-channel groups per voxel (A tile)
  constexpr int BG = BN / 8;
  const int cpg_mask = (1 << g.cpg_shift) - 1;

  for (long long vb = v_begin; vb < v_end; vb += KV) {
    // ---- stage A: KV voxels x BM channels, stored As[ch][v]
    for (int e = tid; e < KV * AG; e += 256) {
      const int v = e / AG, cg = e - v * AG;
      const long long vox = vb + v;
      V8<T> val;
      if (vox < v_end && row0 + cg * 8 < g.Ca) val.load(A + vox * g.lda + row0 + cg * 8);
      else val.zero();
#pragma unroll
      for (int j = 0; j < 8; ++j) As[(cg * 8 + j) * LDS_ROW + v] = from_f<T>(val.get(j));
    }
    // ---- stage B: KV voxels x BN gathered columns, stored Bs[col][v]
    for (int e = tid; e < KV * BG; e += 256) {
      const int v = e / BG, cg = e - v * BG;
      const long long vox = vb + v;
      const int kgi = (col0 >> 3) + cg;
      V8<T> val;
      bool ok = vox < v_end && kgi * 8 < g.Ncols;
      long long src = vox;
      int c8 = kgi;
      if (ok && MODE == MODE_CONV3) {
        const int t = kgi >> g.cpg_shift;
        c8 = kgi & cpg_mask;
        const int x = (int)(vox % g.W);
        long long q = vox / g.W;
        const int y = (int)(q % g.H);
        q /= g.H;
        const int z = (int)(q % g.D);
        int dz, dy, dx;
        tap_delta(t, dz, dy, dx);
        ok = (unsigned)(z + dz) < (unsigned)g.D && (unsigned)(y + dy) < (unsigned)g.H &&
             (unsigned)(x + dx) < (unsigned)g.W;
        src = vox + ((long long)dz * g.H + dy) * g.W + dx;
      } else if (ok && MODE == MODE_CONVT_DGRAD) {
        const int t = kgi >> g.cpg_shift;
        c8 = kgi & cpg_mask;
        const int x = (int)(vox % g.W);
        long long q = vox / g.W;
        const int y = (int)(q % g.H);
        q /= g.H;
        const int z = (int)(q % g.D);
        const long long n = q / g.D;
        src = ((n * 2LL * g.D + 2 * z + (t >> 2)) * 2LL * g.H + 2 * y + ((t >> 1) & 1)) * 2LL * g.W + 2 * x + (t & 1);
      }
      if (ok) val.load(B + src * g.ldb + c8 * 8);
      else val.zero();
#pragma unroll
      for (int j = 0; j < 8; ++j) Bs[(cg * 8 + j) * LDS_ROW + v] = from_f<T>(val.get(j));
    }
    __syncthreads();
    // ---- MFMA over the staged KV voxels
#pragma unroll
    for (int kk = 0; kk < KV; kk += 32) {
      V8<T> af[RM], bfr[RN];
#pragma unroll
      for (int i = 0; i < RM; ++i)
        af[i].load(&As[(wm * RM * 16 + i * 16 + (lane & 15)) * LDS_ROW + kk + (lane >> 4) * 8]);
#pragma unroll
      for (int j = 0; j < RN; ++j)
        bfr[j].load(&Bs[(wn * RN * 16 + j * 16 + (lane & 15)) * LDS_ROW + kk + (lane >> 4) * 8]);
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j) mfma_step<T>(acc[i][j], af[i], bfr[j]);
    }
    __syncthreads();
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
}

// part[ks][row][col] -> torch-layout gradient (fixed-order sum over ks).
//   CONV3 : grad[co][ci][tap]    row=co, col = tap*Cin_pad + ci, ci < Cin_real
//   POINT : grad[co][ci]         row=co, col = ci
//   CONVT : grad[ci][co][tap]    row=ci, col = tap*Cout + co
struct WReduceArgs {
  const float* part;
  float* grad;
  int Ca, Ncols, ksplit;
  int cpad, creal;    // per-tap channel count in cols (padded) and real count
  int ntap;           // 27 (CONV3), 1 (POINT), 8 (CONVT)
  int accumulate;
};

__global__ void wgrad_reduce_kernel(WReduceArgs g, int mode) {
  long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)g.Ca * g.creal * g.ntap;
  if (idx >= total) return;
  // idx enumerates the torch layout [row][c_real][tap]
  const int t = (int)(idx % g.ntap);
  long long q = idx / g.ntap;
  const int c = (int)(q % g.creal);
  const int row = (int)(q / g.creal);
  const int col = t * g.cpad + c;
  const long long stride = (long long)g.Ca * g.Ncols;
  float v = 0.f;
  const float* p = g.part + (long long)row * g.Ncols + col;
  for (int k = 0; k < g.ksplit; ++k) v += p[k * stride];
  if (g.accumulate) g.grad[idx] += v;
  else g.grad[idx] = v;
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

__global__ void colsum_reduce_kernel(const float* __restrict__ part, int nblk, int C, float* __restrict__ out,
                                     int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float v = 0.f;
  for (int b = 0; b < nblk; ++b) v += part[(long long)b * C + c];
  if (accumulate) out[c] += v;
  else out[c] = v;
}

// ------------------------------------------------------------ weight pack
// dst[kgi][col][j] (T), KGp x Cpad x 8, from fp32 torch-layout weights.
//   0 CONV3_FWD  : W[Co][Ci][27]; kgi = tap*(Cip/8)+c8, col = co, ci = c8*8+j
//   1 CONV3_DGRAD: kgi = tap*(Co/8)+c8, col = ci, co = c8*8+j, tap' = 26-tap
//   2 POINT_FWD  : W[Co][Ci]; kgi = c8, col = co, ci = c8*8+j
//   3 POINT_DGRAD: kgi = c8, col = ci, co = c8*8+j
//   4 CONVT_FWD  : W[Ci][Co][8]; kgi = c8 (ci), col = tap*Co + co
//   5 CONVT_DGRAD: kgi = tap*(Co/8)+c8, col = ci, co = c8*8+j
struct PackArgs {
  const float* w;
  void* dst;
  int Co, Ci, Cip;  // Cip: padded input channels (multiple of 8) for CONV3_FWD
  int KG, KGp, Cpad;
};

template <typename T>
__global__ void pack_weight_kernel(PackArgs g, int mode) {
  long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)g.KGp * g.Cpad * 8;
  if (idx >= total) return;
  const int j = (int)(idx & 7);
  const long long q = idx >> 3;
  const int col = (int)(q % g.Cpad);
  const int kgi = (int)(q / g.Cpad);
  float v = 0.f;
  if (kgi < g.KG) {
    switch (mode) {
      case 0: {
        const int cpg = g.Cip >> 3, t = kgi / cpg, ci = (kgi % cpg) * 8 + j, co = col;
        if (co < g.Co && ci < g.Ci) v = g.w[((long long)co * g.Ci + ci) * 27 + t];
      } break;
      case 1: {
        const int cpg = g.Co >> 3, t = kgi / cpg, co = (kgi % cpg) * 8 + j, ci = col;
        if (ci < g.Ci) v = g.w[((long long)co * g.Ci + ci) * 27 + (26 - t)];
      } break;
      case 2: {
        const int ci = kgi * 8 + j, co = col;
        if (co < g.Co && ci < g.Ci) v = g.w[(long long)co * g.Ci + ci];
      } break;
      case 3: {
        const int co = kgi * 8 + j, ci = col;
        if (ci < g.Ci && co < g.Co) v = g.w[(long long)co * g.Ci + ci];
      } break;
      case 4: {
        const int ci = kgi * 8 + j;
        const int t = col / g.Co, co = col % g.Co;
        if (t < 8 && ci < g.Ci) v = g.w[((long long)ci * g.Co + co) * 8 + t];
      } break;
      case 5: {
        const int cpg = g.Co >> 3, t = kgi / cpg, co = (kgi % cpg) * 8 + j, ci = col;
        if (ci < g.Ci) v = g.w[((long long)ci * g.Co + co) * 8 + t];
      } break;
    }
  }
  reinterpret_cast<T*>(g.dst)[idx] = from_f<T>(v);
}

// ------------------------------------------------------------ host launch
template <typename T, int MODE>
int launch_gemm(GemmArgs g, hipStream_t s) {
  const int Cbig = g.Ncols >= 64;
  dim3 block(256);
  if (!Cbig) {
    // BM=128, BN=32
    dim3 grid(ceil_div(g.M, 128), ceil_div(g.Ncols, 32), g.ksplit);
    hipLaunchKernelGGL((conv_gemm_kernel<T, MODE, 4, 1, 2, 2>), grid, block, 0, s, g);
  } else {
    // BM=128, BN=64
    dim3 grid(ceil_div(g.M, 128), ceil_div(g.Ncols, 64), g.ksplit);
    hipLaunchKernelGGL((conv_gemm_kernel<T, MODE, 2, 2, 4, 2>), grid, block, 0, s, g);
  }
  if (mmseg::check_launch("conv_gemm")) return 1;
  if (g.ksplit > 1) {
    long long total = (long long)g.M * g.Ncols;
    hipLaunchKernelGGL((gemm_splitk_reduce<T, MODE>), dim3(ceil_div(total, 256)), dim3(256), 0, s, g);
    if (mmseg::check_launch("gemm_splitk_reduce")) return 1;
  }
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

template <typename T, int MODE>
int launch_wgrad(WgradArgs g, hipStream_t s) {
  dim3 block(256);
  if (g.Ca % 64 == 0) {
    dim3 grid(ceil_div(g.Ncols, 64), g.Ca / 64, g.ksplit);
    hipLaunchKernelGGL((wgrad_kernel<T, MODE, 2, 2, 2, 2, 64>), grid, block, 0, s, g);
  } else {
    dim3 grid(ceil_div(g.Ncols, 64), ceil_div(g.Ca, 32), g.ksplit);
    hipLaunchKernelGGL((wgrad_kernel<T, MODE, 1, 4, 2, 1, 64>), grid, block, 0, s, g);
  }
  return mmseg::check_launch("wgrad");
}

}  // namespace

// =================================================================== C ABI
extern "C" {

// Pack fp32 torch-layout weights into the MFMA B-operand layout [KGp][Cpad][8].
int mmseg_pack_weight(const float* w, void* dst, int mode, int Co, int Ci, int Cip, int KG, int KGp, int Cpad,
                      int dtype, void* stream) {
  PackArgs g{w, dst, Co, Ci, Cip, KG, KGp, Cpad};
  long long total = (long long)KGp * Cpad * 8;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMSEG_BF16)
    hipLaunchKernelGGL(pack_weight_kernel<bf16_t>, dim3(ceil_div(total, 256)), dim3(256), 0, s, g, mode);
  else
    hipLaunchKernelGGL(pack_weight_kernel<float>, dim3(ceil_div(total, 256)), dim3(256), 0, s, g, mode);
  return mmseg::check_launch("pack_weight");
}

// Generic implicit-GEMM: conv3 fwd / dgrad, 1x1, convT fwd / dgrad.
int mmseg_conv_gemm(const void* a, int lda, const void* wpacked, const float* bias, void* out, int ldo,
                    float* splitk_ws, int mode, int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H, int W,
                    int ksplit, int dtype, void* stream) {
  MMSEG_REQUIRE(lda % 8 == 0 && ldo >= 1, "conv_gemm: lda must be a multiple of 8 (got %d)", lda);
  MMSEG_REQUIRE(Cpad >= ((Ncols + (Ncols >= 64 ? 63 : 31)) / (Ncols >= 64 ? 64 : 32)) * (Ncols >= 64 ? 64 : 32),
                "conv_gemm: packed weights must be padded to the column tile (Cpad=%d, Ncols=%d)", Cpad, Ncols);
  MMSEG_REQUIRE(ksplit >= 1, "conv_gemm: ksplit >= 1");
  MMSEG_REQUIRE(ksplit == 1 || splitk_ws != nullptr, "conv_gemm: split-K needs a workspace");
  const int KGp = (KG + 3) & ~3;
  int kps = ((ceil_div(KGp, ksplit) + 3) / 4) * 4;
  ksplit = ceil_div(KGp, kps);
  GemmArgs g{a, lda, wpacked, bias, out, ldo, splitk_ws, M, Ncols, Cpad, KG, cpg_shift, D, H, W, ksplit, kps};
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMSEG_BF16) return launch_gemm_mode<bf16_t>(g, mode, s);
  return launch_gemm_mode<float>(g, mode, s);
}

// Weight-gradient partials: part[ksplit][Ca][Ncols] (fp32).
int mmseg_wgrad(const void* a, int lda, const void* b, int ldb, float* part, int mode, int Ca, int Ncols,
                int cpg_shift, long long V, int D, int H, int W, int ksplit, int dtype, void* stream) {
  MMSEG_REQUIRE(Ca % 8 == 0, "wgrad: rows (%d) must be a multiple of 8", Ca);
  MMSEG_REQUIRE(Ncols % 8 == 0, "wgrad: cols (%d) must be a multiple of 8", Ncols);
  long long vps = ((V + ksplit - 1) / ksplit + 63) / 64 * 64;
  ksplit = (int)((V + vps - 1) / vps);
  WgradArgs g{a, lda, b, ldb, part, Ca, Ncols, cpg_shift, V, D, H, W, ksplit, vps};
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
int mmseg_wgrad_splits(long long V, int ksplit) {
  long long vps = ((V + ksplit - 1) / ksplit + 63) / 64 * 64;
  return (int)((V + vps - 1) / vps);
}

int mmseg_wgrad_reduce(const float* part, float* grad, int Ca, int Ncols, int ksplit, int cpad, int creal, int ntap,
                       int accumulate, void* stream) {
  WReduceArgs g{part, grad, Ca, Ncols, ksplit, cpad, creal, ntap, accumulate};
  long long total = (long long)Ca * creal * ntap;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, g, 0);
  return mmseg::check_launch("wgrad_reduce");
}

// Bias gradient: out[c] (+)= sum_v dy[v][c]; part must hold nblk*C floats.
int mmseg_colsum(const void* dy, int ld, int C, long long V, float* part, int nblk, float* out, int accumulate,
                 int dtype, void* stream) {
  MMSEG_REQUIRE(C % 8 == 0 && C / 8 <= 256, "colsum: C=%d must be a multiple of 8 and <= 2048", C);
  long long vps = (V + nblk - 1) / nblk;
  nblk = (int)((V + vps - 1) / vps);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMSEG_BF16)
    hipLaunchKernelGGL(colsum_partial_kernel<bf16_t>, dim3(nblk), dim3(256), 0, s, (const bf16_t*)dy, ld, C, V, vps,
                       part);
  else
    hipLaunchKernelGGL(colsum_partial_kernel<float>, dim3(nblk), dim3(256), 0, s, (const float*)dy, ld, C, V, vps,
                       part);
  if (mmseg::check_launch("colsum_partial")) return 1;
  hipLaunchKernelGGL(colsum_reduce_kernel, dim3(ceil_div(C, 256)), dim3(256), 0, s, part, nblk, C, out, accumulate);
  return mmseg::check_launch("colsum_reduce");
}

}  // extern "C"
