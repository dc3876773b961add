// Fused Swin window attention (MONAI WindowAttention core, SwinUNETR via the
// reference's swin_unetr.py:80-96): per (window, head) block, scores, the
// relative-position bias, the shifted-window mask, softmax and P.V stay in
// registers / LDS — no materialised N x N score or probability tensors.  bf16
// storage, head_dim <= 16 (padded to the 16-deep MFMA K), N <= 352 tokens.
//
//   fwd   : S^T = K Q^T (v_mfma_f32_16x16x16_bf16: each lane then holds four
//           consecutive keys of ONE query, which is exactly the A-operand
//           layout P needs for O = P V), bias + mask; pass 1 over the key
//           tiles takes the row max / sum, pass 2 recomputes the scores and
//           accumulates O = P V; the row log-sum-exp is kept for the backward.
//   bwd_kv: per key tile, over all query tiles: S and dP = dO V^T recomputed
//           in the [query][key] layout, whose transposed A operand gives
//           dV += P^T dO and dK += scale dS^T Q without shuffles.
//   bwd_q : per query tile, over all key tiles: S^T / dP^T in the forward
//           layout, dQ += scale dS K, and dS written [B][h][N][ldn] for the
//           bias-table gradient (mmseg_relpos_table_grad).
// Two backward passes keep every sum inside one wave (fixed order): no atomics.
// The relative-position index is computed from the token coordinates in the
// module's full window (MONAI indexes relative_position_index[:n, :n] for a
// smaller window, i.e. keeps the full window's numbering), the mask from
// per-window region labels (MONAI compute_mask: -100 across regions).
#include "mmseg_common.h"

namespace {

constexpr int NPMAX = 352;            // tokens per window, padded to 16
constexpr int TP = NPMAX + 8;         // pitch of the [16][tokens] transposed images (720 B: conflict-free)
constexpr int TMAX = 2197;            // (2*7-1)^3 bias-table rows
constexpr int NTMAX = NPMAX / 16;
constexpr int WAVES = 8;               // waves per block (one (window, head) each)
typedef short s4 __attribute__((ext_vector_type(4)));

struct WinAttnArgs {
  const bf16_t* qkv;     // [B*N][3C]
  const bf16_t* O;       // [B*N][C] forward output (bwd)
  const bf16_t* dO;      // [B*N][C] (bwd)
  bf16_t* out;           // fwd: O [B*N][C]; bwd: dqkv [B*N][3C]
  float* lse;            // [B*heads][NPMAX]
  bf16_t* dS;            // bwd_q: [B][heads][N][ldn]
  const float* table;    // [heads][T] (the module's [T][heads] table transposed: one contiguous row per head)
  const uint8_t* region; // [nw][N] or null (no mask)
  int B, N, C, heads, hd, nw, T, ldn;
  int w0, w1, w2;        // the module's full window
  float scale;
  int mixall;            // 1: every window takes the mixed-region score code (the A/B form; 0 in the engine)
  int swz;               // XCD-aware block order (on): a window's heads / query groups,
                         // which stage the same qkv rows (a head's 32-B slice of each), run on one XCD and share its L2
};

// windows of 337..352 tokens (MONAI's 7^3 = 343) take the FULL instantiations: the key-tile loops run to a
// compile-time 22, so the per-tile `kt < nt` guards and their selects around every score update disappear
// (MMSEG_WINATTN_FULL=0: the runtime-bound forms)
int knob_i(const char* name, int dflt);
inline bool wa_full(const WinAttnArgs& a) {
  return ((a.N + 15) & ~15) == NPMAX && knob_i("MMSEG_WINATTN_FULL", 1) != 0;
}

__device__ __forceinline__ int wa_block(const WinAttnArgs& a) {
  return a.swz ? xcd_swizzle((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
}

__device__ __forceinline__ s4 ld4(const bf16_t* p) { return *reinterpret_cast<const s4*>(p); }

// The transposed operand of a token-contracting product from a row image [tokens][16] (ds_read_b64_tr_b16): each
// 16-lane group reads a 4-token x 16-dim block, lane (q = (lane & 15) >> 2, p4 = lane & 3) addressing its token q,
// dims 4 p4 .. +3; lane r16 then holds dim r16 of the 4 tokens -- what the [16][tokens] transposed images held, with
// no transposed copy staged (the per-element LDS stores of that copy were a large share of the staging).
typedef __attribute__((address_space(3))) s4 lds_s4;
__device__ __forceinline__ s4 ld4t(const bf16_t (*rows)[16], int t0) {
  const int lane = threadIdx.x & 63;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(&rows[t0 + ((lane & 15) >> 2)][4 * (lane & 3)]));
}

__device__ __forceinline__ s4 pack4(float a, float b, float c, float d) {
  typedef __bf16 b4 __attribute__((ext_vector_type(4)));
  b4 v = {(bf16_t)a, (bf16_t)b, (bf16_t)c, (bf16_t)d};
  return __builtin_bit_cast(s4, v);
}

__device__ __forceinline__ f32x4 mma(s4 a, s4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}

// relative-position table row of tokens (n, m) in the full window's numbering:
// ((dz + w0-1)(2w1-1) + dy + w1-1)(2w2-1) + dx + w2-1 = code(n) - code(m) + code_off with
// code(n) = (z (2w1-1) + y)(2w2-1) + x, so a per-token code staged in LDS gives the row with one subtraction
// Padding tokens (n >= N) take token 0's code, so every lookup code(n) - code(m) + code_off stays inside the table
// (a real pair's difference): the r05 backward kernels compute those scores unmasked (their probability is zeroed
// by lse = +inf, or the score gradient by a select), and a lookup past the staged table read stale LDS.
__device__ __forceinline__ void stage_codes(int* code, const WinAttnArgs& a, int np) {
  for (int n = threadIdx.x; n < np; n += blockDim.x) {
    const int m = n < a.N ? n : 0;
    const int z = m / (a.w1 * a.w2), y = (m / a.w2) % a.w1, x = m % a.w2;
    code[n] = (z * (2 * a.w1 - 1) + y) * (2 * a.w2 - 1) + x;
  }
}
__device__ __forceinline__ int code_off(const WinAttnArgs& a) {
  return ((a.w0 - 1) * (2 * a.w1 - 1) + (a.w1 - 1)) * (2 * a.w2 - 1) + (a.w2 - 1);
}

// shared operand staging of one (window, head): rows [NPMAX][16] and/or transposed [16][TP]
struct Stage {
  int b, h, N, np;
};

__device__ __forceinline__ void stage_rows(bf16_t (*dst)[16], const bf16_t* src, int ld, int col0, const Stage& s,
                                           int hd, bf16_t (*dstT)[TP]) {
  // thread per (token, 8-channel half); zeros past N and past hd.  SU items per thread per pass, all their loads
  // issued before the first LDS store (one global round trip per pass instead of one per item)
  constexpr int SU = 2;
  for (int e0 = threadIdx.x; e0 < s.np * 2; e0 += SU * blockDim.x) {
    V8<bf16_t> v[SU];
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      const int e = e0 + u * blockDim.x;
      const int n = e >> 1, half = e & 1;
      if (e < s.np * 2 && n < s.N && half * 8 < hd) {
        if (hd >= half * 8 + 8) {
          v[u].load(src + (long long)(s.b * s.N + n) * ld + col0 + half * 8);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            v[u].set(j, half * 8 + j < hd ? (float)src[(long long)(s.b * s.N + n) * ld + col0 + half * 8 + j] : 0.f);
        }
      } else {
        v[u].zero();
      }
    }
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      const int e = e0 + u * blockDim.x;
      if (e >= s.np * 2) break;
      const int n = e >> 1, half = e & 1;
      if (dst) v[u].store(&dst[n][half * 8]);
      if (dstT) {
#pragma unroll
        for (int j = 0; j < 8; ++j) dstT[half * 8 + j][n] = v[u].v[j];
      }
    }
  }
}

// the head's relative-position table row (times mul) into LDS: TU loads per thread in flight (a 7^3 window's
// 2,197-entry table is one pass of 512 threads)
__device__ __forceinline__ void stage_table_m(float* tab, const float* row, int T, float mul) {
  constexpr int TU = 5;
  for (int t0 = threadIdx.x; t0 < T; t0 += TU * blockDim.x) {
    float v[TU];
#pragma unroll
    for (int u = 0; u < TU; ++u) {
      const int tt = t0 + u * blockDim.x;
      v[u] = tt < T ? row[tt] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < TU; ++u) {
      const int tt = t0 + u * blockDim.x;
      if (tt < T) tab[tt] = v[u] * mul;
    }
  }
}

__device__ __forceinline__ void stage_table(float* tab, const WinAttnArgs& a, int h) {
  stage_table_m(tab, a.table + (long long)h * a.T, a.T, 1.f);
}

// the window's region labels (shifted windows) into LDS; returns whether they differ within the window -- only the
// windows along the far faces of the shifted grid mix regions (271 of stage 0's 1,000), the others need no mask.
// Every thread of the block must call it (block-wide vote).
__device__ __forceinline__ bool stage_region(uint8_t* reg, const WinAttnArgs& a, int b) {
  if (!a.region) return false;
  const uint8_t* r = a.region + (long long)(b % a.nw) * a.N;
  const uint8_t r0 = r[0];
  int mixed = 0;
  for (int n = threadIdx.x; n < NPMAX; n += blockDim.x) {
    const uint8_t v = n < a.N ? r[n] : 0;
    reg[n] = v;
    mixed |= (n < a.N && v != r0) ? 1 : 0;
  }
  return __syncthreads_or(mixed) != 0;
}

// ------------------------------------------------------ forward, one pass
// (r05; replaced the r04 two-pass kernel, which recomputed S^T and exp for P V.)  A query tile's whole score row stays in
// registers (22 key tiles x 4 keys per lane = 88 VGPRs), so the scores, their bias / mask and the exponentials are
// computed ONCE instead of twice (the two-pass form recomputed S^T and exp for P V): the kernel was VALU-issue-bound
// at ~50 VALU instructions per MFMA (r05a SQ counters).  Scores are taken in the log2 domain (the table and the scale
// pre-multiplied by log2 e, so a score is one FMA and its exponential one v_exp_f32), P V runs on the full-rate
// 16x16x32 MFMA (two key tiles per instruction, keys permuted identically in P and V), and O is divided by the row
// sum after the product (4 multiplies per lane instead of one per score).  The stored lse is the natural-log one the
// backward expects.
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

__device__ __forceinline__ bf16x8 cat44(s4 a, s4 b) {
  typedef short s8 __attribute__((ext_vector_type(8)));
  const s8 t = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, t);
}

template <bool FULL>
__global__ __launch_bounds__(512) void winattn_fwd1_kernel(WinAttnArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t Qs[NPMAX][16];
  __shared__ __attribute__((aligned(16))) bf16_t Ks[NPMAX][16];
  // (V stays a transposed [16][tokens] image here: the transposed reads of a row image took this kernel from 126 to
  // 130 VGPRs, past the 4-waves-per-SIMD budget)
  __shared__ __attribute__((aligned(16))) bf16_t Vt[16][TP];
  __shared__ float tab[TMAX];
  __shared__ __attribute__((aligned(16))) int code[NPMAX];
  __shared__ __attribute__((aligned(16))) uint8_t reg[NPMAX];
  const int bh = wa_block(a), b = bh / a.heads, h = bh % a.heads;
  const int np = FULL ? NPMAX : (a.N + 15) & ~15, nt = FULL ? NTMAX : np / 16;   // FULL: 22 key tiles, compile-time
  const Stage st{b, h, a.N, np};
  const int C3 = 3 * a.C, hoff = h * a.hd;
  stage_rows(Qs, a.qkv, C3, hoff, st, a.hd, nullptr);
  stage_rows(Ks, a.qkv, C3, a.C + hoff, st, a.hd, nullptr);
  stage_rows(nullptr, a.qkv, C3, 2 * a.C + hoff, st, a.hd, Vt);
  {
    stage_table_m(tab, a.table + (long long)h * a.T, a.T, LOG2E);
  }
  stage_codes(code, a, np);
  const bool rmix = stage_region(reg, a, b);
  __syncthreads();
  const float* ctab = tab + code_off(a);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const float sc2 = a.scale * LOG2E, pen2 = 100.0f * LOG2E;
  const s4 z4 = {0, 0, 0, 0};
#pragma unroll 1   // (one query tile's score row live at a time: with FULL the trip count is known)
  for (int qt = wave; qt < nt; qt += WAVES) {
    const int q = qt * 16 + r16;
    const s4 bq = ld4(&Qs[q][4 * g4]);
    const bool qv = q < a.N;
    const float* tq = ctab + code[q];
    const uint32_t rq = reg[q];
    float v[NTMAX][4];
    float mx = -INFINITY;
    // the score row, instantiated for mixed-region windows and for the rest (no per-score mask compare or select)
    auto scores = [&](auto mixc) __attribute__((always_inline)) {
      constexpr bool MIX = decltype(mixc)::value;
#pragma unroll
      for (int kt = 0; kt < NTMAX; ++kt) {
        if (kt < nt) {
          const f32x4 acc = mma(ld4(&Ks[kt * 16 + r16][4 * g4]), bq, (f32x4){0.f, 0.f, 0.f, 0.f});
          const int k0 = kt * 16 + 4 * g4;
          const int4 ck = *reinterpret_cast<const int4*>(code + k0);
          const uint32_t rk = MIX ? *reinterpret_cast<const uint32_t*>(reg + k0) : 0u;
          const int c[4] = {ck.x, ck.y, ck.z, ck.w};
          const bool last = kt == nt - 1;   // (wave-uniform) only the last key tile holds keys past N
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float t = fmaf(acc[r], sc2, tq[-c[r]]);
            if constexpr (MIX) {
              if (((rk >> (8 * r)) & 255u) != rq) t -= pen2;
            }
            if (last && k0 + r >= a.N) t = -INFINITY;
            v[kt][r] = t;
            mx = fmaxf(mx, t);
          }
        }
        if constexpr (FULL) __builtin_amdgcn_sched_barrier(0);   // one key tile's loads in flight at a time
      }
    };
    if (rmix || a.mixall)
      scores(std::true_type{});
    else
      scores(std::false_type{});
    // (a padding query's row is finite -- its table codes are token 0's -- and is never stored: no select)
#pragma unroll
    for (int o = 16; o <= 32; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    float sum = 0.f;
#pragma unroll
    for (int kt = 0; kt < NTMAX; ++kt) {
      if (kt < nt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = __builtin_amdgcn_exp2f(v[kt][r] - mx);   // exp2(-inf) = 0
          v[kt][r] = p;
          sum += p;
        }
      }
    }
#pragma unroll
    for (int o = 16; o <= 32; o <<= 1) sum += __shfl_xor(sum, o, 64);
    if (g4 == 0 && qv) a.lse[(long long)bh * NPMAX + q] = (mx + __builtin_amdgcn_logf(sum)) * LN2;
    const float inv = sum > 0.f ? 1.f / sum : 0.f;
    f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c2 = 0; c2 < NTMAX / 2; ++c2) {
      const int k0 = 2 * c2;
      if (k0 < nt) {
        const bool hi = k0 + 1 < nt;
        const s4 pa = pack4(v[k0][0], v[k0][1], v[k0][2], v[k0][3]);
        const s4 pb = hi ? pack4(v[k0 + 1][0], v[k0 + 1][1], v[k0 + 1][2], v[k0 + 1][3]) : z4;
        const s4 va = ld4(&Vt[r16][k0 * 16 + 4 * g4]);
        const s4 vb = hi ? ld4(&Vt[r16][(k0 + 1) * 16 + 4 * g4]) : z4;
        o = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cat44(pa, pb), cat44(va, vb), o, 0, 0, 0);
      }
    }
    float ir[4];   // 1 / row sum of query 4 g4 + r (held by lane 4 g4 + r): shuffled with every lane active
#pragma unroll
    for (int r = 0; r < 4; ++r) ir[r] = __shfl(inv, 4 * g4 + r, 64);
    if (r16 < a.hd) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qq = qt * 16 + 4 * g4 + r;
        if (qq < a.N) a.out[(long long)(b * a.N + qq) * a.C + hoff + r16] = (bf16_t)(o[r] * ir[r]);
      }
    }
  }
}

// sum_d dO[row][d] O[row][d] of one head (fp32, d in order): head_dim 16 / 8 from 16-B vector loads issued
// together (a scalar loop over head_dim waited on each 2-B load in turn), any other head_dim element-wise
__device__ __forceinline__ float dot_dO_O(const WinAttnArgs& a, long long base) {
  float d = 0.f;
  if (a.hd == 16 || a.hd == 8) {
    V8<bf16_t> g0, g1, o0, o1;
    g0.load(a.dO + base);
    o0.load(a.O + base);
    if (a.hd == 16) {
      g1.load(a.dO + base + 8);
      o1.load(a.O + base + 8);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) d += g0.get(j) * o0.get(j);
    if (a.hd == 16) {
#pragma unroll
      for (int j = 0; j < 8; ++j) d += g1.get(j) * o1.get(j);
    }
    return d;
  }
  for (int j = 0; j < a.hd; ++j) d += (float)a.dO[base + j] * (float)a.O[base + j];
  return d;
}

// D[q] = sum_d dO[q][d] O[q][d] of this head (fp32), staged into LDS
__device__ __forceinline__ void stage_D(float* Dq, const WinAttnArgs& a, const Stage& s) {
  for (int n = threadIdx.x; n < s.np; n += blockDim.x) {
    float d = 0.f;
    if (n < s.N) d = dot_dO_O(a, (long long)(s.b * s.N + n) * a.C + s.h * a.hd);
    Dq[n] = d;
  }
}

constexpr int QB_TILES = 8;                        // query tiles per block (one per wave) of the query pass

// ----------------------------------------------- backward, r05 forms
// (r05; replaced the r04 kernels.)  Key pass: dV, dK; query pass: dQ and the dS summed over a group of wpg windows on
// chip (the bias-table gradient then folds B / wpg window sums instead of B bf16 score gradients), with what the VALU-issue-bound loops spent
// per score cut: scores in the log2 domain (table and scale pre-multiplied by log2 e, lse staged as lse * log2 e,
// one FMA + one v_exp_f32 per probability); in the key pass invalid queries carry lse = +inf (p = 0 with no select)
// and invalid keys need no mask (their dV / dK rows are never stored); the products that contract over tokens
// (dV, dK over queries; dQ over keys) run on the 16x16x32 MFMA, two token tiles per instruction with the tokens
// permuted identically in both operands.
__device__ __forceinline__ f32x4 mma32(s4 a0, s4 a1, s4 b0, s4 b1, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(cat44(a0, a1), cat44(b0, b1), c, 0, 0, 0);
}

template <bool FULL>
__global__ __launch_bounds__(512) void winattn_bwd_kv2_kernel(WinAttnArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t Qs[NPMAX][16];
  __shared__ __attribute__((aligned(16))) bf16_t Ks[NPMAX][16];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[NPMAX][16];
  __shared__ __attribute__((aligned(16))) bf16_t dOs[NPMAX][16];
  __shared__ float tab[TMAX];
  __shared__ __attribute__((aligned(16))) float lse2[NPMAX];
  __shared__ __attribute__((aligned(16))) float Dq[NPMAX];
  __shared__ __attribute__((aligned(16))) int code[NPMAX];
  __shared__ __attribute__((aligned(16))) uint8_t reg[NPMAX];
  const int bh = wa_block(a), b = bh / a.heads, h = bh % a.heads;
  const int np = FULL ? NPMAX : (a.N + 15) & ~15, nt = FULL ? NTMAX : np / 16;   // FULL: 22 key tiles, compile-time
  const Stage st{b, h, a.N, np};
  const int C3 = 3 * a.C, hoff = h * a.hd;
  stage_rows(Qs, a.qkv, C3, hoff, st, a.hd, nullptr);
  stage_rows(Ks, a.qkv, C3, a.C + hoff, st, a.hd, nullptr);
  stage_rows(Vs, a.qkv, C3, 2 * a.C + hoff, st, a.hd, nullptr);
  stage_rows(dOs, a.dO, a.C, hoff, st, a.hd, nullptr);
  {
    stage_table_m(tab, a.table + (long long)h * a.T, a.T, LOG2E);
  }
  stage_codes(code, a, np);
  const bool rmix = stage_region(reg, a, b);
  stage_D(Dq, a, st);
  for (int n = threadIdx.x; n < np; n += blockDim.x)
    lse2[n] = n < a.N ? a.lse[(long long)bh * NPMAX + n] * LOG2E : INFINITY;
  __syncthreads();
  const float* ctab = tab + code_off(a);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const float sc2 = a.scale * LOG2E, pen2 = 100.0f * LOG2E;
  const s4 z4 = {0, 0, 0, 0};
  for (int kt = wave; kt < nt; kt += WAVES) {
    const int key = kt * 16 + r16;
    const s4 bk = ld4(&Ks[key][4 * g4]);
    const s4 bv = ld4(&Vs[key][4 * g4]);
    const float* tk = ctab - code[key];
    const uint32_t rk = reg[key];
    f32x4 dk = {0.f, 0.f, 0.f, 0.f}, dv = {0.f, 0.f, 0.f, 0.f};
    // instantiated for mixed-region windows and for the rest (no per-score mask compare or select)
    auto pairs = [&](auto mixc) __attribute__((always_inline)) {
      constexpr bool MIX = decltype(mixc)::value;
      for (int qt = 0; qt < nt; qt += 2) {
        s4 pp[2], dd[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int qq = qt + u;
          if (qq < nt) {
            const f32x4 sc = mma(ld4(&Qs[qq * 16 + r16][4 * g4]), bk, (f32x4){0.f, 0.f, 0.f, 0.f});   // S[q][key]
            const f32x4 dp = mma(ld4(&dOs[qq * 16 + r16][4 * g4]), bv, (f32x4){0.f, 0.f, 0.f, 0.f}); // dP[q][key]
            const int q0 = qq * 16 + 4 * g4;
            const int4 cq = *reinterpret_cast<const int4*>(code + q0);
            const uint32_t rq = MIX ? *reinterpret_cast<const uint32_t*>(reg + q0) : 0u;
            const float4 l4 = *reinterpret_cast<const float4*>(lse2 + q0);
            const float4 d4 = *reinterpret_cast<const float4*>(Dq + q0);
            const int c[4] = {cq.x, cq.y, cq.z, cq.w};
            const float lq[4] = {l4.x, l4.y, l4.z, l4.w}, dq4[4] = {d4.x, d4.y, d4.z, d4.w};
            float p[4], ds[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float t = fmaf(sc[r], sc2, tk[c[r]]);
              if constexpr (MIX) {
                if (((rq >> (8 * r)) & 255u) != rk) t -= pen2;
              }
              p[r] = __builtin_amdgcn_exp2f(t - lq[r]);
              ds[r] = p[r] * (dp[r] - dq4[r]);
            }
            pp[u] = pack4(p[0], p[1], p[2], p[3]);
            dd[u] = pack4(ds[0], ds[1], ds[2], ds[3]);
          } else {
            pp[u] = z4;
            dd[u] = z4;
          }
        }
        const bool hi = qt + 1 < nt;
        const s4 o0 = ld4t(dOs, qt * 16 + 4 * g4), o1 = hi ? ld4t(dOs, (qt + 1) * 16 + 4 * g4) : z4;
        const s4 q0 = ld4t(Qs, qt * 16 + 4 * g4), q1 = hi ? ld4t(Qs, (qt + 1) * 16 + 4 * g4) : z4;
        dv = mma32(pp[0], pp[1], o0, o1, dv);
        dk = mma32(dd[0], dd[1], q0, q1, dk);
      }
    };
    if (rmix || a.mixall)
      pairs(std::true_type{});
    else
      pairs(std::false_type{});
    if (r16 < a.hd) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int kk = kt * 16 + 4 * g4 + r;
        if (kk < a.N) {
          bf16_t* row = a.out + (long long)(b * a.N + kk) * C3;
          row[a.C + hoff + r16] = (bf16_t)(dk[r] * a.scale);
          row[2 * a.C + hoff + r16] = (bf16_t)dv[r];
        }
      }
    }
  }
}

// LDS-DMA image of one window for the grouped query pass (double-buffered): each source in its own 1-KB-aligned
// run of 16-B chunks (a wave-instruction moves 64 chunks from ONE buffer resource), chunk c of a run at byte 16 c.
//   K, V: [NPMAX][16] bf16 rows (chunk 2 n + half)      11 instructions each
//   Q, dO, O: the block's 128 queries, [128][16]          4 each
//   lse: [128] f32 (32 chunks)                           1
// Invalid chunks (tokens / queries >= N, the upper 8 dims when head_dim = 8) read through the out-of-range offset
// and land as zeros, as the register staging wrote them.  (The region labels are not DMA'd: a window's row starts
// at byte w N, which a 16-B buffer load cannot address unaligned; one byte per thread, loaded during the previous
// window and stored before its barrier.)
struct QbImg {
  static constexpr int K = 0, V = 11, Q = 22, DO = 26, O = 30, L = 34, NI = 35;   // in 1-KB instructions
  static constexpr int BYTES = NI * 1024;
};

template <bool FULL>
__global__ __launch_bounds__(512) void winattn_bwd_qb2_kernel(WinAttnArgs a, int wpg, int nqg, float* dsum) {
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  __shared__ __attribute__((aligned(16))) char img[2][QbImg::BYTES];
  __shared__ float Dq[2][QB_TILES * 16];
  __shared__ __attribute__((aligned(16))) uint8_t regs[2][NPMAX];
  __shared__ float tab[TMAX];
  __shared__ __attribute__((aligned(16))) int code[NPMAX];
  const int blk = wa_block(a), qg = blk % nqg, h = (blk / nqg) % a.heads, wg = blk / (nqg * a.heads);
  const int np = FULL ? NPMAX : (a.N + 15) & ~15, nt = FULL ? NTMAX : np / 16;   // FULL: 22 key tiles, compile-time
  const int q0 = qg * QB_TILES * 16;
  const int C3 = 3 * a.C, hoff = h * a.hd;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const int qt = qg * QB_TILES + wave;
  const int q = qt * 16 + r16;
  const bool qv = q < a.N;
  {
    stage_table_m(tab, a.table + (long long)h * a.T, a.T, LOG2E);
  }
  stage_codes(code, a, np);
  const float* ctab = tab + code_off(a);
  const float sc2 = a.scale * LOG2E, pen2 = 100.0f * LOG2E;
  const s4 z4 = {0, 0, 0, 0};
  float acc[NTMAX][4];
#pragma unroll
  for (int kt = 0; kt < NTMAX; ++kt)
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[kt][r] = 0.f;
  const int b0 = wg * wpg, b1 = b0 + wpg < a.B ? b0 + wpg : a.B;

  // the DMA of window b into image `buf`.  Wave w issues instructions m = w, w + 8, ... (waves 0-3 five, 4-7 four);
  // instruction m fills 1-KB slot qb_slot(m) of the image: waves 0-3 fetch the dO AND the O rows of the same 32
  // queries (m = 24 + j, 32 + j), so each computes those queries' D = dO . O from its own landed chunks (its vmcnt
  // orders them) before the window's barrier -- no extra barrier, no staging registers.
  const wd_rsrc_t rq_qkv = wd_rsrc(a.qkv, (uint32_t)((long long)a.B * a.N * C3 * 2));
  const wd_rsrc_t rq_do = wd_rsrc(a.dO, (uint32_t)((long long)a.B * a.N * a.C * 2));
  const wd_rsrc_t rq_o = wd_rsrc(a.O, (uint32_t)((long long)a.B * a.N * a.C * 2));
  const wd_rsrc_t rq_l = wd_rsrc(a.lse, (uint32_t)((long long)a.B * a.heads * NPMAX * 4));
  const int wv = __builtin_amdgcn_readfirstlane(wave);   // (wave-uniform: every source / slot choice is scalar)
  auto issue = [&](int buf, int b) __attribute__((always_inline)) {
    const uint32_t lbase = (uint32_t)(uintptr_t)(lds_ptr_t)(&img[buf][0]);
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      int m = wv + 8 * k;
      // (opaque per call: the per-lane offsets below are recomputed per window instead of hoisted out of the window
      // loop for every (k, source) pair the compiler cannot rule out -- that kept ~30 VGPRs live and spilled)
      asm volatile("" : "+s"(m));
      if (m == 31 || m >= 36) continue;   // (31: no source -- the region labels are not DMA'd)
      if (m < 22) {   // K / V rows of the window's tokens: slots 0-21
        const uint32_t lds = lbase + m * 1024;
        const int c = (m < QbImg::V ? m : m - QbImg::V) * 64 + lane, n = c >> 1, half = c & 1;
        const bool ok = n < a.N && half * 8 < a.hd;
        const int col = (m < QbImg::V ? a.C : 2 * a.C) + hoff + half * 8;
        wd_dma16(lds, ok ? (uint32_t)(((b * a.N + n) * C3 + col) * 2) : WD_OOB, rq_qkv);
      } else if (m < 24 || (m >= 28 && m < 30)) {   // Q rows of the block's queries: slots 22-25
        const int j = m < 24 ? m - 22 : m - 26;
        const uint32_t lds = lbase + (QbImg::Q + j) * 1024;
        const int c = j * 64 + lane, n = c >> 1, half = c & 1, qq = q0 + n;
        const bool ok = qq < a.N && half * 8 < a.hd;
        wd_dma16(lds, ok ? (uint32_t)(((b * a.N + qq) * C3 + hoff + half * 8) * 2) : WD_OOB, rq_qkv);
      } else if (m < 28 || m >= 32) {   // dO (m 24-27) / O (m 32-35) rows of queries 32 j .. 32 j + 31
        const bool isdo = m < 28;
        const int j = isdo ? m - 24 : m - 32;
        const uint32_t lds = lbase + ((isdo ? QbImg::DO : QbImg::O) + j) * 1024;
        const int c = j * 64 + lane, n = c >> 1, half = c & 1, qq = q0 + n;
        const bool ok = qq < a.N && half * 8 < a.hd;
        wd_dma16(lds, ok ? (uint32_t)(((b * a.N + qq) * a.C + hoff + half * 8) * 2) : WD_OOB, isdo ? rq_do : rq_o);
      } else {   // m == 30: lse of the block's queries (entries past N are masked when read)
        const int bh = b * a.heads + h;
        wd_dma16(lbase + QbImg::L * 1024, lane < 32 ? (uint32_t)((bh * NPMAX + q0 + 4 * lane) * 4) : WD_OOB, rq_l);
      }
    }
  };
  // D = dO . O (dot_dO_O's arithmetic) of the 32 queries whose dO / O rows this wave fetched into `buf`, after its
  // vmcnt wait; into Dq[buf] for the next window's multiply
  auto dots = [&](int buf) __attribute__((always_inline)) {
    if (wv < 4 && lane < 32) {
      const int n = 32 * wv + lane;
      const bf16_t(*dOs)[16] = reinterpret_cast<const bf16_t(*)[16]>(&img[buf][QbImg::DO * 1024]);
      const bf16_t(*Os)[16] = reinterpret_cast<const bf16_t(*)[16]>(&img[buf][QbImg::O * 1024]);
      float d = 0.f;
      if (q0 + n < a.N) {
        V8<bf16_t> g0, o0;
        g0.load(&dOs[n][0]);
        o0.load(&Os[n][0]);
#pragma unroll
        for (int j = 0; j < 8; ++j) d += g0.get(j) * o0.get(j);
        if (a.hd == 16) {
          V8<bf16_t> g1, o1;
          g1.load(&dOs[n][8]);
          o1.load(&Os[n][8]);
#pragma unroll
          for (int j = 0; j < 8; ++j) d += g1.get(j) * o1.get(j);
        }
      }
      Dq[buf][n] = d;
    }
  };
  const int tid = threadIdx.x;
  auto region_byte = [&](int b) __attribute__((always_inline)) -> uint8_t {   // stage_region's value of token tid
    return (a.region && tid < a.N) ? a.region[(long long)(b % a.nw) * a.N + tid] : (uint8_t)0;
  };
  if (b0 < b1) {
    if (tid < NPMAX) regs[0][tid] = region_byte(b0);
    __syncthreads();   // table / codes / first labels staged
    issue(0, b0);
    __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0): this wave's chunks landed
    dots(0);
    __syncthreads();
  }
  for (int b = b0; b < b1; ++b) {
    const int cur = (b - b0) & 1;
    if (b + 1 < b1) issue(cur ^ 1, b + 1);   // (the other image was last read before the previous barrier)
    const uint8_t nreg = b + 1 < b1 ? region_byte(b + 1) : (uint8_t)0;   // (stored before this window's barrier)
    const char* I = img[cur];
    const bf16_t(*Ks)[16] = reinterpret_cast<const bf16_t(*)[16]>(I + QbImg::K * 1024);
    const bf16_t(*Vs)[16] = reinterpret_cast<const bf16_t(*)[16]>(I + QbImg::V * 1024);
    const bf16_t(*Qs)[16] = reinterpret_cast<const bf16_t(*)[16]>(I + QbImg::Q * 1024);
    const bf16_t(*dOs)[16] = reinterpret_cast<const bf16_t(*)[16]>(I + QbImg::DO * 1024);
    const float* Ls = reinterpret_cast<const float*>(I + QbImg::L * 1024);
    const uint8_t* reg = regs[cur];
    // windows that mix shifted regions (stage_region's vote, per wave over the landed labels)
    bool rmix = false;
    if (a.region) {
      const uint8_t r0 = reg[0];
      int mixed = 0;
      for (int n = lane; n < a.N; n += 64) mixed |= reg[n] != r0;
      rmix = __any(mixed);
    }
    if (qt < nt) {
      const int ql = wave * 16 + r16;
      const s4 bq = ld4(&Qs[ql][4 * g4]);
      const s4 bdo = ld4(&dOs[ql][4 * g4]);
      const float dq_ = Dq[cur][ql];
      const float lq = (qv ? Ls[ql] : 0.f) * LOG2E;
      const float* tq = ctab + code[q];
      const uint32_t rq = a.region ? reg[q] : 0u;
      f32x4 dq = {0.f, 0.f, 0.f, 0.f};
      // instantiated for mixed-region windows and for the rest (no per-score mask compare or select)
      auto tiles = [&](auto mixc) __attribute__((always_inline)) {
        constexpr bool MIX = decltype(mixc)::value;
#pragma unroll
        for (int k2 = 0; k2 < NTMAX / 2; ++k2) {
          s4 dd[2];
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const int kt = 2 * k2 + u;
            if (kt < nt) {
              const f32x4 sc = mma(ld4(&Ks[kt * 16 + r16][4 * g4]), bq, (f32x4){0.f, 0.f, 0.f, 0.f});
              const f32x4 dp = mma(ld4(&Vs[kt * 16 + r16][4 * g4]), bdo, (f32x4){0.f, 0.f, 0.f, 0.f});
              const int k0 = kt * 16 + 4 * g4;
              const int4 ck = *reinterpret_cast<const int4*>(code + k0);
              const uint32_t rk = MIX ? *reinterpret_cast<const uint32_t*>(reg + k0) : 0u;
              const int c[4] = {ck.x, ck.y, ck.z, ck.w};
              float ds[4];
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                float t = fmaf(sc[r], sc2, tq[-c[r]]);
                if constexpr (MIX) {
                  if (((rk >> (8 * r)) & 255u) != rq) t -= pen2;
                }
                const float p = __builtin_amdgcn_exp2f(t - lq);
                // (an explicitly rounded product: with `acc += p * (...)` the compiler may contract into an FMA
                // or not depending on the instantiation, and the summed gradient must be the same bits in both)
                ds[r] = __fmul_rn(p, dp[r] - dq_);
                if (kt == nt - 1 && k0 + r >= a.N) ds[r] = 0.f;   // keys past N (only in the last tile)
                acc[kt][r] += ds[r];
              }
              dd[u] = pack4(ds[0], ds[1], ds[2], ds[3]);
            } else {
              dd[u] = z4;
            }
          }
          const int kt0 = 2 * k2;
          if (kt0 < nt) {
            const bool hi = kt0 + 1 < nt;
            const s4 k0v = ld4t(Ks, kt0 * 16 + 4 * g4), k1v = hi ? ld4t(Ks, (kt0 + 1) * 16 + 4 * g4) : z4;
            dq = mma32(dd[0], dd[1], k0v, k1v, dq);
          }
        }
      };
      if (rmix || a.mixall)
        tiles(std::true_type{});
      else
        tiles(std::false_type{});
      if (r16 < a.hd) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int qq = qt * 16 + 4 * g4 + r;
          if (qq < a.N) a.out[(long long)(b * a.N + qq) * C3 + hoff + r16] = (bf16_t)(dq[r] * a.scale);
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0): this wave's chunks of window b + 1 landed
    if (b + 1 < b1) {
      dots(cur ^ 1);
      if (tid < NPMAX) regs[cur ^ 1][tid] = nreg;
    }
    __syncthreads();
  }
  if (qt < nt && qv) {
    float* row = dsum + (((long long)wg * a.heads + h) * a.N + q) * a.ldn;
#pragma unroll
    for (int kt = 0; kt < NTMAX; ++kt) {
      const int k0 = kt * 16 + 4 * g4;
      if (kt < nt && k0 < a.ldn) {
        if (k0 + 3 < a.ldn) {
          *reinterpret_cast<float4*>(row + k0) = make_float4(acc[kt][0], acc[kt][1], acc[kt][2], acc[kt][3]);
        } else {
          for (int r = 0; r < 4 && k0 + r < a.ldn; ++r) row[k0 + r] = acc[kt][r];
        }
      }
    }
  }
}

// bwd_q in the r05 form (one window per block, dS written per window in bf16 for mmseg_relpos_table_grad): the
// same per-score arithmetic and MFMA order as winattn_bwd_qb2_kernel, so dQ is bitwise the summed path's.
template <bool FULL>
__global__ __launch_bounds__(512) void winattn_bwd_q2_kernel(WinAttnArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t Qs[NPMAX][16];
  __shared__ __attribute__((aligned(16))) bf16_t Ks[NPMAX][16];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[NPMAX][16];
  __shared__ __attribute__((aligned(16))) bf16_t dOs[NPMAX][16];
  __shared__ float tab[TMAX];
  __shared__ __attribute__((aligned(16))) float lse2[NPMAX];
  __shared__ __attribute__((aligned(16))) float Dq[NPMAX];
  __shared__ __attribute__((aligned(16))) int code[NPMAX];
  __shared__ __attribute__((aligned(16))) uint8_t reg[NPMAX];
  const int bh = wa_block(a), b = bh / a.heads, h = bh % a.heads;
  const int np = FULL ? NPMAX : (a.N + 15) & ~15, nt = FULL ? NTMAX : np / 16;   // FULL: 22 key tiles, compile-time
  const Stage st{b, h, a.N, np};
  const int C3 = 3 * a.C, hoff = h * a.hd;
  stage_rows(Qs, a.qkv, C3, hoff, st, a.hd, nullptr);
  stage_rows(Ks, a.qkv, C3, a.C + hoff, st, a.hd, nullptr);
  stage_rows(Vs, a.qkv, C3, 2 * a.C + hoff, st, a.hd, nullptr);
  stage_rows(dOs, a.dO, a.C, hoff, st, a.hd, nullptr);
  {
    stage_table_m(tab, a.table + (long long)h * a.T, a.T, LOG2E);
  }
  stage_codes(code, a, np);
  const bool rmix = stage_region(reg, a, b);
  stage_D(Dq, a, st);
  for (int n = threadIdx.x; n < np; n += blockDim.x) lse2[n] = n < a.N ? a.lse[(long long)bh * NPMAX + n] * LOG2E : 0.f;
  __syncthreads();
  const float* ctab = tab + code_off(a);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, g4 = lane >> 4;
  const float sc2 = a.scale * LOG2E, pen2 = 100.0f * LOG2E;
  const s4 z4 = {0, 0, 0, 0};
  for (int qt = wave; qt < nt; qt += WAVES) {
    const int q = qt * 16 + r16;
    const s4 bq = ld4(&Qs[q][4 * g4]);
    const s4 bdo = ld4(&dOs[q][4 * g4]);
    const float lq = lse2[q], dq_ = Dq[q];
    const float* tq = ctab + code[q];
    const uint32_t rq = reg[q];
    f32x4 dq = {0.f, 0.f, 0.f, 0.f};
    bf16_t* dsrow = a.dS + ((long long)bh * a.N + q) * a.ldn;
#pragma unroll
    for (int k2 = 0; k2 < NTMAX / 2; ++k2) {
      s4 dd[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int kt = 2 * k2 + u;
        if (kt < nt) {
          const f32x4 sc = mma(ld4(&Ks[kt * 16 + r16][4 * g4]), bq, (f32x4){0.f, 0.f, 0.f, 0.f});
          const f32x4 dp = mma(ld4(&Vs[kt * 16 + r16][4 * g4]), bdo, (f32x4){0.f, 0.f, 0.f, 0.f});
          const int k0 = kt * 16 + 4 * g4;
          const int4 ck = *reinterpret_cast<const int4*>(code + k0);
          const uint32_t rk = rmix ? *reinterpret_cast<const uint32_t*>(reg + k0) : 0u;
          const int c[4] = {ck.x, ck.y, ck.z, ck.w};
          float ds[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float t = fmaf(sc[r], sc2, tq[-c[r]]);
            if (rmix && ((rk >> (8 * r)) & 255u) != rq) t -= pen2;
            const float p = __builtin_amdgcn_exp2f(t - lq);
            ds[r] = __fmul_rn(p, dp[r] - dq_);   // (as the grouped query pass: the same dQ bits)
            if (kt == nt - 1 && k0 + r >= a.N) ds[r] = 0.f;
          }
          dd[u] = pack4(ds[0], ds[1], ds[2], ds[3]);
          if (q < a.N) {
            if (k0 + 3 < a.ldn) {
              *reinterpret_cast<s4*>(dsrow + k0) = dd[u];
            } else {
              typedef __bf16 b4 __attribute__((ext_vector_type(4)));
              const b4 v = __builtin_bit_cast(b4, dd[u]);
              for (int r = 0; r < 4 && k0 + r < a.ldn; ++r) dsrow[k0 + r] = v[r];
            }
          }
        } else {
          dd[u] = z4;
        }
      }
      const int kt0 = 2 * k2;
      if (kt0 < nt) {
        const bool hi = kt0 + 1 < nt;
        const s4 k0v = ld4t(Ks, kt0 * 16 + 4 * g4), k1v = hi ? ld4t(Ks, (kt0 + 1) * 16 + 4 * g4) : z4;
        dq = mma32(dd[0], dd[1], k0v, k1v, dq);
      }
    }
    if (r16 < a.hd) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qq = qt * 16 + 4 * g4 + r;
        if (qq < a.N) a.out[(long long)(b * a.N + qq) * C3 + hoff + r16] = (bf16_t)(dq[r] * a.scale);
      }
    }
  }
}

// windows per block of winattn_bwd_qb: about two resident blocks per CU over (window group, head, query group)
int qb_windows_per_group(int B, int N, int heads) {
  const int nt = ((N + 15) & ~15) / 16, nqg = (nt + QB_TILES - 1) / QB_TILES;
  int nwg = (512 + heads * nqg - 1) / (heads * nqg);
  if (nwg > B) nwg = B;
  if (nwg < 1) nwg = 1;
  return (B + nwg - 1) / nwg;
}

int knob_i(const char* name, int dflt) {
  const char* v = getenv(name);
  return v ? atoi(v) : dflt;
}

int check_args(const WinAttnArgs& a) {
  MMSEG_REQUIRE(a.N >= 1 && a.N <= NPMAX && a.hd >= 1 && a.hd <= 16 && a.hd % 8 == 0 && a.C == a.heads * a.hd &&
                    a.T <= TMAX && a.T == (2 * a.w0 - 1) * (2 * a.w1 - 1) * (2 * a.w2 - 1) &&
                    (a.region == nullptr || a.nw >= 1),
                "winattn: N <= %d, head_dim 8 or 16, table rows <= %d", NPMAX, TMAX);
  return 0;
}

}  // namespace

extern "C" {

long long mmseg_winattn_lse_floats(int B, int heads) { return (long long)B * heads * NPMAX; }

int mmseg_winattn_fwd(const void* qkv, int B, int N, int C, int heads, const float* table, int T, int w0, int w1,
                      int w2, const uint8_t* region, int nw, float scale, void* O, float* lse, void* stream) {
  WinAttnArgs a{(const bf16_t*)qkv, nullptr, nullptr, (bf16_t*)O, lse, nullptr, table, region,
                B, N, C, heads, C / heads, nw, T, 0, w0, w1, w2, scale};
  a.swz = 1;      // XCD-aware block order (r05 (iii))
  a.mixall = 0;   // the region compare only for windows that mix shifted regions (r05 (vi))
  if (check_args(a)) return 1;
  mmseg::note_kernel("winattn_fwd1_kernel");
  if (wa_full(a))
    MMSEG_LAUNCH(winattn_fwd1_kernel<true>, dim3(B * heads), dim3(64 * WAVES), 0, (hipStream_t)stream, a);
  else
    MMSEG_LAUNCH(winattn_fwd1_kernel<false>, dim3(B * heads), dim3(64 * WAVES), 0, (hipStream_t)stream, a);
  return mmseg::check_launch("winattn_fwd");
}

int mmseg_winattn_bwd(const void* qkv, const void* O, const void* dO, const float* lse, int B, int N, int C, int heads,
                      const float* table, int T, int w0, int w1, int w2, const uint8_t* region, int nw, float scale,
                      void* dqkv, void* dS, int ldn, void* stream) {
  WinAttnArgs a{(const bf16_t*)qkv, (const bf16_t*)O, (const bf16_t*)dO, (bf16_t*)dqkv, const_cast<float*>(lse),
                (bf16_t*)dS, table, region, B, N, C, heads, C / heads, nw, T, ldn, w0, w1, w2, scale};
  a.swz = 1;      // XCD-aware block order (r05 (iii))
  a.mixall = 0;   // the region compare only for windows that mix shifted regions (r05 (vi))
  if (check_args(a)) return 1;
  MMSEG_REQUIRE(ldn >= N && ldn % 8 == 0, "winattn_bwd: ldn >= N, multiple of 8");
  hipStream_t s = (hipStream_t)stream;
  if (wa_full(a)) MMSEG_LAUNCH(winattn_bwd_kv2_kernel<true>, dim3(B * heads), dim3(64 * WAVES), 0, s, a);
  else MMSEG_LAUNCH(winattn_bwd_kv2_kernel<false>, dim3(B * heads), dim3(64 * WAVES), 0, s, a);
  if (mmseg::check_launch("winattn_bwd_kv")) return 1;
  if (wa_full(a)) MMSEG_LAUNCH(winattn_bwd_q2_kernel<true>, dim3(B * heads), dim3(64 * WAVES), 0, s, a);
  else MMSEG_LAUNCH(winattn_bwd_q2_kernel<false>, dim3(B * heads), dim3(64 * WAVES), 0, s, a);
  mmseg::note_kernel("winattn_bwd_kv2_kernel");
  return mmseg::check_launch("winattn_bwd_q");
}

// Window groups of mmseg_winattn_bwd_sum (0: too few windows per group to pay -- use mmseg_winattn_bwd).
int mmseg_winattn_sum_groups(int B, int N, int heads) {
  const int wpg = qb_windows_per_group(B, N, heads);
  return wpg >= 4 ? (B + wpg - 1) / wpg : 0;
}

// mmseg_winattn_bwd with the score gradient summed over groups of windows on chip: dsum [groups][heads][N][ldn]
// fp32 (groups = mmseg_winattn_sum_groups(), keys >= N zero) replaces dS [B][heads][N][ldn]; fold it with
// mmseg_relpos_table_grad(dsum, ldn, groups, ..., dtype = f32).  dqkv is bitwise mmseg_winattn_bwd's.
int mmseg_winattn_bwd_sum(const void* qkv, const void* O, const void* dO, const float* lse, int B, int N, int C,
                          int heads, const float* table, int T, int w0, int w1, int w2, const uint8_t* region, int nw,
                          float scale, void* dqkv, float* dsum, int ldn, void* stream) {
  WinAttnArgs a{(const bf16_t*)qkv, (const bf16_t*)O, (const bf16_t*)dO, (bf16_t*)dqkv, const_cast<float*>(lse),
                nullptr, table, region, B, N, C, heads, C / heads, nw, T, ldn, w0, w1, w2, scale};
  a.swz = 1;      // XCD-aware block order (r05 (iii))
  a.mixall = 0;   // the region compare only for windows that mix shifted regions (r05 (vi))
  if (check_args(a)) return 1;
  MMSEG_REQUIRE(ldn >= N && ldn % 8 == 0 && mmseg_winattn_sum_groups(B, N, heads) > 0,
                "winattn_bwd_sum: ldn >= N (multiple of 8) and enough windows (mmseg_winattn_sum_groups)");
  MMSEG_REQUIRE((long long)B * N * 3 * C * 2 < (1LL << 31) && (long long)B * heads * NPMAX * 4 < (1LL << 31),
                "winattn_bwd_sum: the query pass's 32-bit DMA offsets need qkv and lse under 2 GB");
  hipStream_t s = (hipStream_t)stream;
  if (wa_full(a)) MMSEG_LAUNCH(winattn_bwd_kv2_kernel<true>, dim3(B * heads), dim3(64 * WAVES), 0, s, a);
  else MMSEG_LAUNCH(winattn_bwd_kv2_kernel<false>, dim3(B * heads), dim3(64 * WAVES), 0, s, a);
  if (mmseg::check_launch("winattn_bwd_kv")) return 1;
  const int wpg = qb_windows_per_group(B, N, heads);
  const int nt = ((N + 15) & ~15) / 16, nqg = (nt + QB_TILES - 1) / QB_TILES, nwg = (B + wpg - 1) / wpg;
  if (wa_full(a))
    MMSEG_LAUNCH(winattn_bwd_qb2_kernel<true>, dim3(nwg * heads * nqg), dim3(64 * WAVES), 0, s, a, wpg, nqg, dsum);
  else
    MMSEG_LAUNCH(winattn_bwd_qb2_kernel<false>, dim3(nwg * heads * nqg), dim3(64 * WAVES), 0, s, a, wpg, nqg, dsum);
  mmseg::note_kernel("winattn_bwd_kv2_kernel");
  return mmseg::check_launch("winattn_bwd_qb");
}

}  // extern "C"
