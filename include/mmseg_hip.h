/*
 * mmseg_hip.h — C ABI of libmmseg_hip.so, the MI355X (gfx950) kernels of the
 * multimodal organ segmentation training step.
 *
 * The reference (wittyseok/multimodal-organ-segmentation) has no FFI: its hot
 * path is implicit ATen ops reached through torch.nn modules.  Each entry
 * point below replaces the ATen op(s) named in its comment (reference
 * file:line); the Python mirror of the reference API
 * (multimodal-organ-segmentation_amd/models, /trainer) binds them with ctypes
 * (INTEGRATION.md shows the binding).
 *
 * Conventions
 *   - Every function returns 0 on success, non-zero on failure; the message of
 *     the last failure on the calling thread is mmseg_last_error().  No C++
 *     exception crosses the ABI.
 *   - All pointers are device pointers owned by the caller (torch caching
 *     allocator); kernels never allocate or free.  Workspaces are sized by the
 *     *_ws_floats() queries.
 *   - `stream` is a hipStream_t; every call is enqueue-only (no host sync), so
 *     call sequences can be captured into a hipGraph.
 *   - Activations are NDHWC: element (n, v, c) at base[(n*V + v)*ld + c],
 *     V = D*H*W, ld >= C (ld > C: a slot of a wider concat buffer).
 *   - dtype: 0 = fp32 storage (parity mode), 1 = bf16 storage; all
 *     accumulation is fp32.  Reductions are fixed-order (deterministic).
 */
#ifndef MMSEG_HIP_H
#define MMSEG_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------- plumbing */
const char* mmseg_last_error(void);
/* Name of the main kernel the last conv/wgrad entry point launched on this thread (for the per-kernel timer). */
const char* mmseg_last_kernel(void);
int mmseg_abi_version(void);
/* Launch timing for the per-kernel timer (bench.py's roofline): between begin and end every kernel of the
 * library is launched with hipExtLaunchKernelGGL start / stop events, which the runtime stamps from the
 * dispatch itself (the kernel's own begin / end, as rocprofv3's kernel trace reports them).  After the work
 * has completed, mmseg_timing_get(i) gives launch i's duration and its launch-site kernel expression. */
int mmseg_timing_begin(void);
int mmseg_timing_end(void);
long long mmseg_timing_count(void);
int mmseg_timing_get(long long i, float* ms, const char** name);

/* --------------------------------------------------------- GEMM family */
/* Gather modes: 0 CONV3 (3x3x3, pad 1), 1 POINT (1x1x1), 2 CONVT_FWD (k2 s2,
 * output scatter), 3 CONVT_DGRAD (k2 s2, child gather). */

/* fp32 torch-layout weights -> MFMA B-operand layout [KGp][Cpad][8].
 * mode 0/1: Conv3d W[Co][Ci][3][3][3] fwd / dgrad (flipped, transposed)
 * mode 2/3: 1x1 Conv3d W[Co][Ci] fwd / dgrad
 * mode 4/5: ConvTranspose3d W[Ci][Co][2][2][2] fwd / dgrad
 * mode 6/7: the mode 1 / mode 5 data-gradient images over Cip >= Co zero-padded output channels (the
 *           reduction of a layer whose Co is not 8 x a power of two, e.g. SwinUNETR's 48 / 96 / 384)
 * Replaces the weight reads of nn.Conv3d / nn.ConvTranspose3d (unet.py:26-27, 95, 163). */
int mmseg_pack_weight(const float* w, void* dst, int mode, int Co, int Ci, int Cip, int KG, int KGp, int Cpad,
                      int dtype, void* stream);

/* Batched form: one launch packs every layer of a model from a device table of
 * descriptors {w, dst, mode, Co, Ci, Cip, KG, KGp, Cpad, pad, begin} (mmseg_pack_desc_bytes() each). */
/* Batched pack of every 3^3 conv of a model, both images (forward + data-gradient) from one read.
 * descs: device array of n records {w, wf, wd|NULL, Co, Ci, Cip, Cpad, Cpad_d, block_begin, Cop, pad}
 * (Cop: the data-gradient image's padded output-channel count, pack mode 6; 0 = Co)
 * (mmseg_pack3_desc_bytes() each), layer l owning blocks [block_begin, +Co/8*ceil(Ci/32)).
 * The images must be zero-initialised once (padding entries are never written). */
int mmseg_pack3_desc_bytes(void);
int mmseg_pack_conv3_batched(const void* descs, int n, int nblocks, int dtype, void* stream);
int mmseg_pack_desc_bytes(void);
int mmseg_pack_weights_batched(const void* descs, int n, long long total, int dtype, void* stream);

/* CONV3 data gradient (ksplit 1, no bias) that also writes the InstanceNorm-backward partial sums of its output:
 * the output is dy of an InstanceNorm + ReLU with pre-norm input inx (pitch ldinx) and statistics inmean /
 * inrstd [N][Ncols]; inpart [N][mmseg_conv3_dgrad_in_chunks()][Ncols][2] = (sum g, sum g xhat), g = dy [xhat > 0],
 * the layout mmseg_instnorm_bwd_part reads.  bf16, the brick5 kernel's shapes only (chunks 0 otherwise). */
int mmseg_conv3_dgrad_in_chunks(int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H, int W, int lda,
                                int ldo, int dtype);
int mmseg_conv3_dgrad_in(const void* a, int lda, const void* wpacked, void* out, int ldo, int M, int Ncols, int Cpad,
                         int KG, int cpg_shift, int D, int H, int W, const void* inx, int ldinx, const float* inmean,
                         const float* inrstd, float* inpart, int dtype, void* stream);
/* Split count the CONV3 kernel choice wants for this shape (value-returning, not a status): the caller
 * allocates ksplit*M*Ncols fp32 of split-K workspace and passes ksplit to mmseg_conv_gemm. */
int mmseg_conv3_splits(int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H, int W, int lda, int ldo,
                       int dtype);
/* Implicit-GEMM forward / data-gradient convolution on MFMA.
 * Replaces aten::convolution (fwd) and convolution_backward (grad_input) of
 * Conv3d(k3,p1) unet.py:26-27, ConvTranspose3d(k2,s2) unet.py:95, and the
 * 1x1 projections unet.py:163 / dual_encoder.py:75.  splitk_ws holds
 * ksplit*M*Ncols floats when ksplit > 1. */
int mmseg_conv_gemm(const void* a, int lda, const void* wpacked, const float* bias, void* out, int ldo,
                    float* splitk_ws, int mode, int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H, int W,
                    int ksplit, int dtype, void* stream);

/* First conv of an encoder with Cr <= 8 real input channels (unet.py:26 via unet.py:154-157 / dual_encoder.py:66-70)
 * on the 8-channel packed input (ldx == 8), K = 27*Cr exactly instead of 27*8.  Replaces aten::convolution and
 * convolution_backward (grad_weight, grad_bias) of that layer.  mmseg_stem_ok / _kp / _wgrad_splits return values.
 * Weight gradient: part[ks][Co][KP] + bias_part[ks][Co], summed by mmseg_wgrad_reduce(Ca=Co, Ncols=KP, cpad=creal=Cr,
 * ntap=27). */
int mmseg_stem_ok(int cr, int Co, int D, int H, int W, int ldx, int ldy);
int mmseg_stem_kp(int cr);
int mmseg_stem_wgrad_splits(int N, int D, int H, int W, int want);
int mmseg_stem_fwd(const void* x, int ldx, int cr, const float* w, const float* bias, void* y, int ldy, int N, int D,
                   int H, int W, int Co, int dtype, void* stream);
/* mmseg_stem_fwd that also writes InstanceNorm partials of its output: stats [N][mmseg_stem_stats_bricks()][Co][2]
 * = (mean, M2) of the stored values over each 1x8x8 slice of its 4x8x8 bricks (64 voxels), the input of
 * mmseg_instnorm_stats_bricks(stats, N, Co, slices, 64, ...). */
int mmseg_stem_stats_bricks(int D, int H, int W);
int mmseg_stem_fwd_stats(const void* x, int ldx, int cr, const float* w, const float* bias, void* y, int ldy, int N,
                         int D, int H, int W, int Co, float* stats, int dtype, void* stream);
int mmseg_stem_wgrad(const void* dy, int lddy, const void* x, int ldx, int cr, float* part, float* bias_part, int N,
                     int D, int H, int W, int Co, int ksplit, int dtype, void* stream);
/* mmseg_stem_wgrad whose dy is the gradient of an InstanceNorm + ReLU OUTPUT: the norm's backward (pre-norm
 * input inx with pitch ldinx, statistics inmean / inrstd [N][Co], coefficients incoef [N][Co][2] from
 * mmseg_instnorm_bwd_coef) is applied while staging dy -- the values mmseg_instnorm_bwd would write, bit for bit --
 * so the norm's input gradient is never materialised.  inx null: mmseg_stem_wgrad. */
int mmseg_stem_wgrad_inb(const void* dy, int lddy, const void* x, int ldx, int cr, const void* inx, int ldinx,
                         const float* inmean, const float* inrstd, const float* incoef, float* part, float* bias_part,
                         int N, int D, int H, int W, int Co, int ksplit, int dtype, void* stream);

/* Fused InstanceNorm statistics (unet.py:34 InstanceNorm3d following each Conv3d): when the CONV3 brick kernel
 * for a shape can emit them, mmseg_conv3_stats_bricks returns the bricks per sample (value-returning, 0 = not
 * available) and mmseg_conv_gemm_stats writes stats_part[N][bricks][Ncols][2] = per-brick (mean, M2) of the stored
 * outputs; mmseg_instnorm_stats_bricks turns them into mean / rstd, replacing the statistics pass over the output. */
int mmseg_conv3_stats_bricks(int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H, int W, int lda, int ldo,
                             int dtype);
int mmseg_conv_gemm_stats(const void* a, int lda, const void* wpacked, const float* bias, void* out, int ldo,
                          float* splitk_ws, int mode, int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H,
                          int W, int ksplit, float* stats_part, int dtype, void* stream);
/* mmseg_conv_gemm_stats whose A source holds only cin_real real channels (the rest are channel padding with zero
 * packed weights, e.g. SwinUNETR's 96 / 192 / 384 / 768-channel tensors stored as 128 / 256 / 512 / 1024): the CONV3
 * brick kernels skip the 32-channel K chunks wholly past cin_real.  cin_real = 0: all channels are real.  Replaces
 * the same Conv3d call sites as mmseg_conv_gemm (monai SwinUNETR's UnetResBlock convs). */
int mmseg_conv_gemm_ex(const void* a, int lda, const void* wpacked, const float* bias, void* out, int ldo,
                       float* splitk_ws, int mode, int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H,
                       int W, int ksplit, float* stats_part, int cin_real, int dtype, void* stream);
/* mmseg_conv_gemm_ex (no statistics) with a whole-row output hint: the brick2 conv kernels also write zeros into
 * columns [Ncols, zcols) of the output rows (zcols <= min(ldo, Ncols + 48), multiple of 8; 0 = none), so 48 / 96
 * real columns at pitch 64 / 128 are written in whole 128-B lines; other kernels leave those columns alone. */
int mmseg_conv_gemm_zw(const void* a, int lda, const void* wpacked, const float* bias, void* out, int ldo,
                       float* splitk_ws, int mode, int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H,
                       int W, int ksplit, int cin_real, int zcols, int dtype, void* stream);
int mmseg_instnorm_stats_bricks(const float* part, int N, int C, int nb, int cnt, float eps, float* mean, int mean_ld,
                                float* rstd, void* stream);

/* Weight-gradient partials part[ksplit][Ca][Ncols] (fp32), K = voxels.
 * Replaces convolution_backward (grad_weight) of the same layers; with
 * bias_part != NULL (a = dy) also the grad_bias partials bias_part[ksplit][Ca]. */
int mmseg_wgrad(const void* a, int lda, const void* b, int ldb, float* part, float* bias_part, int mode, int Ca,
                int Ncols, int cpg_shift, long long V, int D, int H, int W, int ksplit, int dtype, void* stream);
/* Split counts mmseg_wgrad will use (value-returning): callers size part[] with them.  For CONV3 the
 * library picks the split of its brick kernels itself; ksplit is then only the caller's workspace cap. */
int mmseg_wgrad_splits(long long V, int ksplit);
int mmseg_wgrad_splits_conv3(long long V, int ksplit, int Ca, int cpg_shift, int D, int H, int W, int lda, int ldb,
                             int dtype);
/* Fixed-order sum of the partials into the torch-layout fp32 gradient. */
int mmseg_wgrad_reduce(const float* part, float* grad, const float* bias_part, float* bias_grad, int Ca, int Ncols,
                       int ksplit, int cpad, int creal, int ntap, int accumulate, void* stream);
/* Weight + bias gradient of a 3^3 Conv3d (convolution_backward grad_weight / grad_bias of unet.py:26-27)
 * straight into the torch-layout fp32 grad[Co][Ci][3][3][3] and bias_grad[Co] (NULL: no bias), = or +=
 * (accumulate).  dy: [V][Co] (ld lddy), x: [V][Cip] (ld ldx), Cip = 8 << cpg_shift >= Ci real channels.
 * The library picks kernel and voxel split; ws holds mmseg_conv3_wgrad_ws_floats() floats (a smaller
 * ws_floats clamps the split; 0 is enough whenever the query returned 0). */
long long mmseg_conv3_wgrad_ws_floats(long long V, int Co, int Cip, int Ci, int cpg_shift, int D, int H, int W,
                                      int lddy, int ldx, int dtype);
int mmseg_conv3_wgrad(const void* dy, int lddy, const void* x, int ldx, float* grad, float* bias_grad, int Co, int Cip,
                      int Ci, int cpg_shift, long long V, int D, int H, int W, float* ws, long long ws_floats,
                      int accumulate, int dtype, void* stream);
/* mmseg_conv_gemm_ex (without fused statistics) with the output columns [split, Ncols) written to a second
 * tensor out2 (row pitch ldo2) as its columns 0..Ncols-split-1 (split, ldo, ldo2 multiples of 8, out2 16-B
 * aligned; not the transposed-conv forward): the decoder's first-conv data gradient writes d(upsampled) and
 * d(skip) as two dense tensors. */
int mmseg_conv_gemm_split(const void* a, int lda, const void* wpacked, const float* bias, void* out, int ldo,
                          void* out2, int ldo2, int split, float* splitk_ws, int mode, int M, int Ncols, int Cpad,
                          int KG, int cpg_shift, int D, int H, int W, int ksplit, int cin_real, int dtype,
                          void* stream);
/* 1x1 GEMM (MODE_POINT, no split-K) with a residual epilogue: out = round(round(A W^T + bias) + res) -- bitwise the
 * GEMM into a temporary followed by mmseg_add(res, temporary, out); res may alias out; ldo, ldres, Ncols multiples
 * of 8, out / res 16-B aligned.  SwinUNETR's residual sums (UnetResBlock dx += d(conv3 branch), MLP x + fc2(.);
 * reference swin_unetr.py:80-96 -> MONAI) without their own pass. */
int mmseg_conv_gemm_res(const void* a, int lda, const void* wpacked, const float* bias, const void* res, int ldres,
                        void* out, int ldo, int M, int Ncols, int Cpad, int KG, int dtype, void* stream);
/* 1x1 GEMM (MODE_POINT, no split-K) with the MLP's GELU (exact erf) in its epilogue: epi 1, out = h = A W^T + bias
 * and gelu_out = gelu(h) (MLPBlock linear1 + GELU); epi 2, out = (A W^T) * gelu'(gelu_in) (linear2's data gradient
 * through the GELU, gelu_in = h) -- bitwise the GEMM followed by mmseg_gelu_fwd / mmseg_gelu_bwd; every buffer at
 * pitch ldo (multiple of 8), 16-B aligned (reference swin_unetr.py:80-96 -> MONAI MLPBlock). */
int mmseg_conv_gemm_gelu(const void* a, int lda, const void* wpacked, const float* bias, void* out, int ldo,
                         const void* gelu_in, void* gelu_out, int epi, int M, int Ncols, int Cpad, int KG, int dtype,
                         void* stream);
/* Deferred InstanceNorm + ReLU of a 3^3 conv's input (the block's conv1 output is never written by its
 * normalisation pass): the input holds the PRE-norm activation and the kernels stage
 * relu((x - mean[n][c]) * rstd[n][c]) rounded to bf16, the values mmseg_instnorm_relu_fwd would write.
 * *_ok return 1 when the shape runs the kernels that support it (brick5 forward, brick2 weight gradient). */
int mmseg_conv3_norm_ok(int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H, int W, int lda, int ldo,
                        int dtype);
int mmseg_conv3_fwd_norm(const void* a, int lda, const float* nmean, const float* nrstd, const void* wpacked,
                         const float* bias, void* out, int ldo, int M, int Ncols, int Cpad, int KG, int cpg_shift,
                         int D, int H, int W, int dtype, void* stream);
/* Mixed bf16/fp8 forward (config c5, "mixed bf16/fp8"): the 3^3 convs the brick kernels take with one 32-channel
 * input chunk run with OCP e4m3 operands and fp32 accumulation.  mmseg_pack_conv3_fp8 writes the e4m3 image of
 * w[co] * s[co], s[co] = 448 / max|w[co]|, and wdq[co] = 1 / s[co]; mmseg_conv3_fwd_fp8 stages the (optionally
 * normalised, as mmseg_conv3_fwd_norm) bf16 input as e4m3 at unit scale and writes bf16.  Replaces the
 * reference's Conv3d forward (unet.py:26-27, 53-60) under its mixed-precision mode. */
int mmseg_conv3_fp8_ok(int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H, int W, int lda, int ldo);
int mmseg_pack_conv3_fp8(const float* w, int Co, int Ci, int Cip, int KGp, int Cpad, void* dst, float* wdq,
                         void* stream);
int mmseg_conv3_fwd_fp8(const void* a, int lda, const float* nmean, const float* nrstd, const void* w8,
                        const float* wdq, const float* bias, void* out, int ldo, int M, int Ncols, int Cpad, int KG,
                        int cpg_shift, int D, int H, int W, void* stream);
int mmseg_conv3_wgrad_norm_ok(long long V, int Co, int Cip, int Ci, int cpg_shift, int D, int H, int W, int lddy,
                              int ldx, int dtype);
int mmseg_conv3_wgrad_norm(const void* dy, int lddy, const void* x, int ldx, const float* nmean, const float* nrstd,
                           float* grad, float* bias_grad, int Co, int Cip, int Ci, int cpg_shift, long long V, int D,
                           int H, int W, float* ws, long long ws_floats, int accumulate, int dtype, void* stream);
/* Grouped forms for `groups` same-shape layers over equal sample groups of one activation tensor (group gi:
 * samples [gi N / groups, (gi + 1) N / groups)), each with its own weights: the M modality encoders' small levels
 * (12^3 / 6^3, runtime-brick kernels) as one launch instead of M.  Replace the same ATen ops as mmseg_conv_gemm_ex /
 * mmseg_conv3_wgrad (reference unet.py:26-27, run once per modality encoder, dual_encoder.py:112-165).
 * conv_gemm_group: group gi reads wpacked + gi * w_gstride (elements) and bias + gi * b_gstride.
 * conv3_wgrad_group: group gi's gradients go to grad + gi * grad_gstride / bias_grad + gi * bias_gstride floats;
 * ws holds mmseg_conv3_wgrad_group_ws_floats() floats; phase as mmseg_conv3_wgrad_ex. */
int mmseg_conv_gemm_group(const void* a, int lda, const void* wpacked, const float* bias, void* out, int ldo,
                          float* splitk_ws, int mode, int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H,
                          int W, int ksplit, int cin_real, int groups, long long w_gstride, int b_gstride, int dtype,
                          void* stream);
int mmseg_conv3_group_ok(int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H, int W, int lda, int ldo,
                         int dtype);
int mmseg_conv3_wgrad_group_ok(long long V, int Co, int Cip, int Ci, int cpg_shift, int D, int H, int W, int lddy,
                               int ldx, int dtype);
int mmseg_conv3_group_splits(int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H, int W, int lda, int ldo,
                             int dtype);
/* conv_gemm_group + the output's per-brick InstanceNorm partials (the runtime-brick epilogue; one split): stats_part
 * [M / (D H W)][conv3_group_stats_bricks()][Ncols][2] (mean, M2), merged by mmseg_instnorm_stats_bricks -- the
 * grouped 48^3 / 24^3 levels' statistics without a pass over the output (reference unet.py:28-29 InstanceNorm). */
int mmseg_conv3_group_stats_bricks(int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H, int W, int lda,
                                   int ldo, int dtype);
int mmseg_conv_gemm_group_stats(const void* a, int lda, const void* wpacked, const float* bias, void* out, int ldo,
                                int mode, int M, int Ncols, int Cpad, int KG, int cpg_shift, int D, int H, int W,
                                int cin_real, int groups, long long w_gstride, int b_gstride, float* stats_part,
                                int dtype, void* stream);
long long mmseg_conv3_wgrad_group_ws_floats(long long V, int Co, int Cip, int Ci, int cpg_shift, int D, int H, int W,
                                            int lddy, int ldx, int groups, int dtype);
int mmseg_conv3_wgrad_group(const void* dy, int lddy, const void* x, int ldx, float* grad, float* bias_grad, int Co,
                            int Cip, int Ci, int cpg_shift, long long V, int D, int H, int W, float* ws,
                            long long ws_floats, int accumulate, int groups, long long grad_gstride,
                            int bias_gstride, int phase, int dtype, void* stream);
/* mmseg_conv3_wgrad (nmean / nrstd: optional deferred norm, as mmseg_conv3_wgrad_norm) in phases: bit 1 runs
 * the weight-gradient kernel, bit 2 the split reduce (3 = both), so the kernel can be timed alone.  Bit 4 with
 * bit 2 defers the reduce: its arguments are queued until mmseg_wgrad_reduce_flush(stream), which sums every
 * queued reduce of that stream in one launch (bitwise the same gradients); the partials (ws) must stay untouched
 * until then. */
int mmseg_wgrad_reduce_flush(void* stream);
/* mmseg_wgrad_reduce queued for the next mmseg_wgrad_reduce_flush on `stream` (part untouched until then) */
int mmseg_wgrad_reduce_defer(const float* part, float* grad, const float* bias_part, float* bias_grad, int Ca,
                             int Ncols, int ksplit, int cpad, int creal, int ntap, int accumulate, void* stream);
int mmseg_wgrad_reduce_pending(void);
int mmseg_wgrad_reduce_discard(void* stream);
/* phase bit 8 (with bit 1): rows [Co - 16, Co) of dy / the gradient are output-channel padding (SwinUNETR's 48 real
 * channels in 64-row tiles): the 64-row LDS-DMA weight-gradient kernel multiplies 48 rows and writes zeros there
 * (other kernels ignore the bit); the real rows are bitwise unchanged. */
int mmseg_conv3_wgrad_ex(const void* dy, int lddy, const void* x, int ldx, const float* nmean, const float* nrstd,
                         float* grad, float* bias_grad, int Co, int Cip, int Ci, int cpg_shift, long long V, int D,
                         int H, int W, float* ws, long long ws_floats, int accumulate, int phase, int dtype,
                         void* stream);
/* Bias gradient out[c] (+)= sum_v dy[v][c] (convolution_backward grad_bias). */
int mmseg_colsum(const void* dy, int ld, int C, long long V, float* part, int nblk, float* out, int accumulate,
                 int dtype, void* stream);
/* out[c] (+)= sum_{b < nblk} part[b][c] in fixed order: the transposed conv's bias gradient from the column-sum
 * partials mmseg_wgrad(MODE_CONVT_DGRAD, bias_part = [ksplit][8 Cout]) emits, with nblk = 8 ksplit. */
int mmseg_colsum_reduce(const float* part, int nblk, int C, float* out, int accumulate, void* stream);

/* ---------------------------------------- InstanceNorm3d + ReLU, MaxPool */
long long mmseg_instnorm_ws_floats(int N, long long V, int C);
/* Per-(n,c) mean / 1/sqrt(var+eps) (nn.InstanceNorm3d unet.py:34-35, biased var).
 * mean[n*mean_ld + c]; rstd may be NULL (channel means only, e.g. AdaptiveAvgPool3d). */
int mmseg_instnorm_stats(const void* x, int ldx, int N, long long V, int C, float eps, float* mean, int mean_ld,
                         float* rstd, float* ws, int dtype, void* stream);
/* y = relu((x - mean) * rstd)  (InstanceNorm3d + ReLU(inplace), unet.py:54-59). */
int mmseg_instnorm_relu_fwd(const void* x, int ldx, void* y, int ldy, int N, long long V, int C, const float* mean,
                            const float* rstd, int dtype, void* stream);
/* mmseg_instnorm_relu_bwd over G modality groups of one combined tensor (N = G x n samples): p1 holds n samples and
 * sample k reads p1 sample k % p1_nmod (p1_nmod = n) -- the fused level's gradient, read once for all G encoders
 * (reference dual_encoder.py:193-195 / 184-186 fusion backward + unet.py:34-35 InstanceNorm + ReLU backward). */
int mmseg_instnorm_relu_bwd_group(const void* x, int ldx, const float* mean, const float* rstd, const void* p1,
                                  int ld1, float scale1, int p1_nmod, const void* pool_dy, int pool_ld,
                                  const uint8_t* pool_idx, void* dx, int lddx, int N, int D, int H, int W, int C,
                                  float* ws, int dtype, void* stream);
/* Backward of InstanceNorm3d + ReLU with dy gathered as
 *   dy = scale1*alpha1[n]*p1 + beta[n][c] + maxpool_bwd(pool_dy, pool_idx)
 * (MaxPool3d backward unet.py:73 and the DualEncoder fusion backward
 * dual_encoder.py:167-199 fused in; any source may be NULL). */
int mmseg_instnorm_relu_bwd(const void* x, int ldx, const float* mean, const float* rstd, const void* p1, int ld1,
                            float scale1, const float* alpha1, int alpha_stride, const float* beta, int beta_stride,
                            const void* pool_dy, int pool_ld, const uint8_t* pool_idx, void* dx, int lddx, int N,
                            int D, int H, int W, int C, float* ws, int dtype, void* stream);
/* Backward of InstanceNorm3d (no affine) with the activation after it folded in: act 0 none, 1 ReLU, 2
 * LeakyReLU(slope); g is the gradient of the activation's OUTPUT, dx that of the norm's input x (MONAI UnetResBlock
 * norms, reference swin_unetr.py:80-96).  part / nchunk: partial sums a producer of g emitted
 * (mmseg_lrelu_bwd_in_part; finalize + apply only) or NULL / 0.  Cw (C <= Cw <= min(2 C, lddx), multiple of 8, or 0
 * = C): dx's channels [C, Cw) are written as zeros (whole-row writes).  ws: mmseg_instnorm_ws_floats. */
int mmseg_instnorm_act_bwd(const void* x, int ldx, const float* mean, const float* rstd, const void* g, int ldg,
                           void* dx, int lddx, int N, int D, int H, int W, int C, int Cw, int act, float slope,
                           const float* part, int nchunk, float* ws, int dtype, void* stream);
/* Chunks per sample of the InstanceNorm-backward partial sums over V voxels x C channels (0: unsupported shape). */
int mmseg_instnorm_part_chunks(long long V, int C);
/* UnetResBlock tail backward, first pass (y = LeakyReLU(IN(xa) + IN(xb)) or LeakyReLU(IN(xa) + residual)):
 * g = dy * (y > 0 ? 1 : slope), stored, and in the same pass the InstanceNorm-backward partial sums of xa (and of xb
 * if non-NULL) over g: pa / pb [N][mmseg_instnorm_part_chunks(V, C)][C][2], the layout mmseg_instnorm_bwd_part
 * finalises and applies.  Bitwise what mmseg_lrelu_bwd + the norms' own partial passes give.  Cw: g's channels
 * [C, Cw) written as zeros (as mmseg_lrelu_bwd). */
int mmseg_lrelu_bwd_in_part(const void* y, int ldy, const void* dy, int lddy, void* g, int ldg, float slope,
                            const void* xa, int lda, const float* ma, const float* ra, float* pa, const void* xb,
                            int ldb, const float* mb, const float* rb, float* pb, int N, long long V, int C, int Cw,
                            int dtype, void* stream);
/* Statistics + normalisation (+ ReLU if relu) in one call: y = [relu]((x - mean) * rstd), mean / rstd written as
 * by mmseg_instnorm_stats (mean_ld == C).  Volumes of <= 4096 voxels per sample take one fused launch (one block
 * per 8-channel group and sample, the 12^3 / 6^3 levels); larger ones the stats + apply passes. */
int mmseg_instnorm_fwd(const void* x, int ldx, void* y, int ldy, int N, long long V, int C, float eps, float* mean,
                       int mean_ld, float* rstd, int relu, float* ws, int dtype, void* stream);
/* The same two without the ReLU (relu = 0): InstanceNorm3d alone, as in the residual
 * norm(query + out) of CrossAttentionFusion (attention_fusion.py:161-162). */
int mmseg_instnorm_apply(const void* x, int ldx, void* y, int ldy, int N, long long V, int C, const float* mean,
                         const float* rstd, int relu, int dtype, void* stream);
int mmseg_instnorm_bwd(const void* x, int ldx, const float* mean, const float* rstd, const void* p1, int ld1,
                       float scale1, const float* alpha1, int alpha_stride, const float* beta, int beta_stride,
                       const void* pool_dy, int pool_ld, const uint8_t* pool_idx, void* dx, int lddx, int N, int D,
                       int H, int W, int C, int relu, float* ws, int dtype, void* stream);
/* mmseg_instnorm_bwd with the partial sums [N][nchunk][C][2] (sum g, sum g * xhat per chunk, g = dy [xhat > 0])
 * already emitted by the producer of dy (mmseg_head_loss_bwd_in): finalize + apply only; ws holds 2 N C floats. */
int mmseg_instnorm_bwd_part(const void* x, int ldx, const float* mean, const float* rstd, const void* p1, int ld1,
                            float scale1, const float* alpha1, int alpha_stride, const float* beta, int beta_stride,
                            const void* pool_dy, int pool_ld, const uint8_t* pool_idx, void* dx, int lddx, int N,
                            int D, int H, int W, int C, int relu, const float* part, int nchunk, float* ws,
                            int dtype, void* stream);
/* The coefficient half of mmseg_instnorm_bwd for dy = p1: coef [N][C][2] = (mean g, mean g xhat), from given
 * partials (part, nchunk; as for mmseg_instnorm_bwd_part) or, part null, from a partial pass (ws:
 * mmseg_instnorm_ws_floats floats).  Its apply half runs inside mmseg_stem_wgrad_inb. */
int mmseg_instnorm_bwd_coef(const void* x, int ldx, const float* mean, const float* rstd, const void* p1, int ld1,
                            int N, int D, int H, int W, int C, int relu, const float* part, int nchunk,
                            float* coef, float* ws, int dtype, void* stream);
/* MaxPool3d(2) forward + argmax (0..7, z-major; first max wins) (unet.py:73). */
int mmseg_maxpool2_fwd(const void* x, int ldx, void* y, int ldy, uint8_t* idx, int N, int D, int H, int W, int C,
                       int dtype, void* stream);
/* The same over relu((x - mean) * rstd) of a PRE-norm x (mean / rstd [N][C]): values and argmax equal pooling
 * the materialised InstanceNorm + ReLU output (rounded to the storage type first), which is never written. */
int mmseg_maxpool2_norm_fwd(const void* x, int ldx, const float* mean, const float* rstd, void* y, int ldy,
                            uint8_t* idx, int N, int D, int H, int W, int C, int dtype, void* stream);

/* ---------------------------------------------------- modality fusion */
/* out = wconst * sum_m src_m (mean / add fusion, dual_encoder.py:184-186,193-195)
 * or sum_m wts[n][m] * src_m (CrossModalAttention weighting, dual_encoder.py:252-254). */
int mmseg_fuse_fwd(const void* const* srcs, const int* lds, int M, float wconst, const float* wts, void* out, int ldo,
                   int N, long long V, int C, int dtype, void* stream);
/* mmseg_fuse_fwd over relu((src_m - mean_m) * rstd_m) of PRE-norm sources (the encoders' last InstanceNorm +
 * ReLU applied on load; means / rstds: M pointers to [N][C] statistics). */
int mmseg_fuse_norm_fwd(const void* const* srcs, const int* lds, const float* const* means, const float* const* rstds,
                        int M, float wconst, const float* wts, void* out, int ldo, int N, long long V, int C,
                        int dtype, void* stream);
/* CrossModalAttention gate: Linear -> ReLU -> Linear -> softmax (dual_encoder.py:226-233). */
int mmseg_attn_gate_fwd(const float* pooled, const float* W1, const float* b1, const float* W2, const float* b2,
                        float* hbuf, float* wts, int N, int MC, int Hd, int M, void* stream);
int mmseg_attn_gate_bwd(const void* const* srcs, const int* lds, int M, const void* dfused, int ldd, int N, long long V,
                        int C, const float* pooled, const float* W1, const float* W2, const float* hbuf,
                        const float* wts, float* beta, float* gW1, float* gb1, float* gW2, float* gb2, int Hd,
                        float* ws, int accumulate, int dtype, void* stream);

/* ------------------------------------------- multi-head cross-attention */
/* CrossAttentionFusion (attention_fusion.py:77-164, unwired in the reference's model factory).
 * Batched NT GEMM on MFMA: C[b][i][j] (+)= alpha * sum_k A[b][i][k] * B[b][j][k] (+ bias[j]), batch index
 * b = outer * inner + in, operand X at X + outer*sX_outer + in*sX_inner, row stride ldX (elements).
 * A/B in the storage dtype (lda, ldb, A/B strides multiples of 8, 16-B aligned; K not a multiple of 8 reads the
 * last 8-group whole, so the row padding up to round_up(K, 8) of A or B must be zero); C fp32 (c_dtype 0) or
 * the storage dtype.  Replaces the 1x1 Conv3d projections (:117-120, :159), einsum("bhdn,bhdm->bhnm")
 * (:147-148), einsum("bhnm,bhdm->bhdn") (:153) and their gradients. */
int mmseg_bgemm_nt(const void* a, long long sa_outer, long long sa_inner, int lda, const void* b, long long sb_outer,
                   long long sb_inner, int ldb, void* c, long long sc_outer, long long sc_inner, int ldc,
                   const float* bias, int batch, int inner, int M, int N, int K, float alpha, int accumulate,
                   int c_dtype, int dtype, void* stream);
/* dst[b][c][r] = src[b][r][c] with dtype conversion (0 fp32, 1 bf16): operand re-layout and the
 * NCDHW fp32 <-> NDHWC module boundary. */
int mmseg_transpose(const void* src, long long s_outer, long long s_inner, int lds, int src_dtype, void* dst,
                    long long d_outer, long long d_inner, int ldd, int dst_dtype, int batch, int inner, int rows,
                    int cols, void* stream);
/* Row softmax of fp32 scores into P (storage dtype), F.softmax(attn, dim=-1) (:149), and its backward
 * dS = P * (dP - rowsum(dP * P)). */
int mmseg_softmax_rows(const float* S, int lds, void* P, int ldp, long long rows, int N, int dtype, void* stream);
int mmseg_softmax_bwd_rows(const void* P, int ldp, const float* dP, int lddp, void* dS, int ldds, long long rows,
                           int N, int dtype, void* stream);

/* Swin window attention (MONAI SwinUNETR WindowAttention, reached from swin_unetr.py:80-96; MONAI absent ->
 * parity unpinned).  relpos_bias: bias[h][n][m] = table[index[n*N+m]][h] (table [T][heads]).
 * softmax_bias_rows: rows = windows*heads*N of fp32 scores S, P = softmax(S + bias[h] + mask[w]) (row
 * padding [N, ldp) of P written as zeros, as by mmseg_softmax_rows / _bwd_rows) with
 * h = (row / N) % heads, w = (row / (N*heads)) % nw (bias / mask may be NULL).
 * relpos_table_grad: dB[h][n][m] = sum_b dS[b][h][n][m] (B window batches, fixed order), then
 * gtable[t][h] (+)= sum over the CSR list offs[t]..offs[t+1] of (n*N+m) entries of dB[h]. */
int mmseg_relpos_bias(const float* table, const int* index, int heads, int N, float* bias, void* stream);
int mmseg_softmax_bias_rows(const float* S, int lds, const float* bias, const float* mask, int nw, int heads, void* P,
                            int ldp, long long rows, int N, int dtype, void* stream);
int mmseg_relpos_table_grad(const void* dS, int ldn, int B, int heads, int N, float* dB, const int* offs,
                            const int* pairs, int T, float* gtable, int accumulate, int dtype, void* stream);

/* Fused window attention core (bf16, head_dim 8 or 16, <= 352 tokens per window): per (window, head),
 * O = softmax(scale q k^T + table[rel(n, m)] (+ -100 across regions)) v with the scores kept on chip.
 * qkv [B*N][3C] (q | k | v, head h at channels h*hd), O [B*N][C], lse [B*heads][352] (row log-sum-exp,
 * mmseg_winattn_lse_floats()), table [heads][T] (the module's [T][heads] bias table transposed) with
 * T = (2w0-1)(2w1-1)(2w2-1) of the module's full window
 * (w0, w1, w2): rel() numbers the tokens in that window, as MONAI's relative_position_index[:N, :N];
 * region [nw][N] uint8 labels of the shifted-window regions of window b % nw, or NULL (no mask).
 * bwd: dqkv [B*N][3C] (every element written) and dS [B][heads][N][ldn] (bf16, keys >= N zero) for
 * mmseg_relpos_table_grad. */
long long mmseg_winattn_lse_floats(int B, int heads);
int mmseg_winattn_fwd(const void* qkv, int B, int N, int C, int heads, const float* table, int T, int w0, int w1,
                      int w2, const uint8_t* region, int nw, float scale, void* O, float* lse, void* stream);
int mmseg_winattn_bwd(const void* qkv, const void* O, const void* dO, const float* lse, int B, int N, int C, int heads,
                      const float* table, int T, int w0, int w1, int w2, const uint8_t* region, int nw, float scale,
                      void* dqkv, void* dS, int ldn, void* stream);
/* winattn_bwd_sum: mmseg_winattn_bwd with the score gradient summed over groups of windows on chip (dqkv bitwise
 * the same): dsum [groups][heads][N][ldn] fp32, groups = mmseg_winattn_sum_groups(B, N, heads) (0 = not worth it,
 * use mmseg_winattn_bwd); fold with mmseg_relpos_table_grad(dsum, ldn, groups, ..., dtype f32). */
int mmseg_winattn_sum_groups(int B, int N, int heads);
int mmseg_winattn_bwd_sum(const void* qkv, const void* O, const void* dO, const float* lse, int B, int N, int C,
                          int heads, const float* table, int T, int w0, int w1, int w2, const uint8_t* region, int nw,
                          float scale, void* dqkv, float* dsum, int ldn, void* stream);

/* ---------------------------------------------------- SwinUNETR tokens */
/* The SwinTransformer stages and UNETR residual blocks of MONAI SwinUNETR (built by the reference's
 * swin_unetr.py:80-96; MONAI absent -> parity unpinned, restated in oracle/swin_oracle.py).  Token
 * tensors are channels-last rows [rows][ld].
 * layernorm_fwd: nn.LayerNorm(C) / F.layer_norm (gamma = beta = NULL: no affine, proj_out); mean / rstd
 *   per row (may be NULL).  layernorm_bwd: dx (+)= (add_dx) the input gradient; dgamma / dbeta (+)=
 *   (accumulate) from per-block partials in ws (mmseg_layernorm_bwd_ws_floats() floats). */
int mmseg_layernorm_fwd(const void* x, int ldx, void* y, int ldy, long long rows, int C, const float* gamma,
                        const float* beta, float eps, float* mean, float* rstd, int dtype, void* stream);
long long mmseg_layernorm_bwd_ws_floats(long long rows, int C);
int mmseg_layernorm_bwd(const void* x, int ldx, const void* dy, int lddy, void* dx, int lddx, long long rows, int C,
                        const float* gamma, const float* mean, const float* rstd, int add_dx, float* dgamma,
                        float* dbeta, int accumulate, float* ws, int dtype, void* stream);
/* nn.GELU() (exact erf) of MLPBlock, and its backward dh = dy * gelu'(h); n % 8 == 0, contiguous. */
int mmseg_gelu_fwd(const void* h, void* y, long long n, int dtype, void* stream);
int mmseg_gelu_bwd(const void* h, const void* dy, void* dh, long long n, int dtype, void* stream);
/* out = a + b (contiguous, n % 8 == 0): the MLP residual of SwinTransformerBlock. */
int mmseg_add(const void* a, const void* b, void* out, long long n, int dtype, void* stream);
/* nn.Dropout(p) at MONAI SwinUNETR's drop_rate sites (swin_unetr.py:87 drop_rate -> pos_drop,
 * WindowAttention proj_drop, MLPBlock drop1/drop2).  y = keep ? x / (1 - p) : 0 over a [rows][C] buffer
 * (in place allowed), keep from a counter hash of (seed, element index) — flat, or NCDHW order when ncdhw
 * (rows = N * V).  The backward is the same call on the gradient with the same seed. */
int mmseg_dropout(const void* x, void* y, long long rows, int C, long long V, int ncdhw, float p, long long seed,
                  int dtype, void* stream);
/* F.pad to the padded grid (Dp, Hp, Wp) + torch.roll(-s) + window_partition -> dst [B*nW][w0*w1*w2][C].
 * window_reverse: the inverse (window_reverse + roll(+s) + crop) onto the real grid, plus add_src
 * (the block's shortcut; NULL: none).  Also the backward of each other. */
int mmseg_window_partition(const void* src, int ldx, int B, int D, int H, int W, int C, int w0, int w1, int w2,
                           int s0, int s1, int s2, int Dp, int Hp, int Wp, void* dst, int dtype, void* stream);
int mmseg_window_reverse(const void* win, int B, int D, int H, int W, int C, int w0, int w1, int w2, int s0, int s1,
                         int s2, int Dp, int Hp, int Wp, const void* add_src, int ld_add, void* dst, int ld_dst,
                         int dtype, void* stream);
/* Legacy PatchMerging sub-grid concat [B, ceil(D/2).., 8C] (odd sides zero padded) and its backward
 * (sum over the slots that read each voxel; voxels no slot reads get 0). */
int mmseg_merge_gather(const void* x, int ldx, int B, int D, int H, int W, int C, void* out, int dtype, void* stream);
int mmseg_merge_scatter(const void* dout, int B, int D, int H, int W, int C, void* dx, int lddx, int dtype,
                        void* stream);
/* PatchEmbed Conv3d(k2, s2) operand: NCDHW fp32 [B][Cin][D][H][W] -> [B*(D/2)(H/2)(W/2)][Kp],
 * column ci*8 + kz*4 + ky*2 + kx (the weight's own flattening), columns >= 8*Cin zero. */
int mmseg_patchify(const float* x, int B, int Cin, int D, int H, int W, int Kp, void* out, int dtype, void* stream);
/* UnetResBlock tail: y = lrelu((a - ma) * ra + R), R = (b - mb) * rb (b normalised), b (identity
 * residual, mb = rb = NULL) or 0 (b = NULL); stats [N][C].  lrelu_bwd: g = dy * (y > 0 ? 1 : slope).
 * Cw (C <= Cw <= min(2 C, output pitch), multiple of 8): the output's channels [C, Cw) are written as zeros, so a
 * row padded past C (48 channels at pitch 64) is written whole -- partial-row writes run at ~60 % of the rate. */
int mmseg_res_apply(const void* a, int lda, const float* ma, const float* ra, const void* b, int ldb, const float* mb,
                    const float* rb, void* y, int ldy, int N, long long V, int C, int Cw, float slope, int dtype,
                    void* stream);
int mmseg_lrelu_bwd(const void* y, int ldy, const void* dy, int lddy, void* g, int ldg, long long rows, int C, int Cw,
                    float slope, int dtype, void* stream);

/* ------------------------------------------------------- device data path */
/* ModalitySpecificNormalize (src/data/transforms.py:362-404) on one channel [V] fp32 in place:
 * kind 0 CT window (lo = center - width/2, hi = center + width/2): clip + (x - lo) / (hi - lo);
 * kind 1 PET: x / max(x) when max > 0; kind 2 MRI/US: (x - mean) / (std + 1e-8), fp64 statistics.
 * ws: mmseg_normalize_ws_bytes() bytes (kinds 1, 2). */
long long mmseg_normalize_ws_bytes(void);
int mmseg_modality_normalize(float* x, long long V, int kind, double lo, double hi, void* ws, void* stream);
/* Resize (transforms.py:215-250): scipy.ndimage.zoom order 1 per channel of src [C][D][H][W] -> dst
 * [C][d][h][w] (corner-aligned, fp64 math), and order 0 for labels (int64 or uint8). */
int mmseg_resize_linear(const float* src, int C, int D, int H, int W, float* dst, int d, int h, int w, void* stream);
int mmseg_resize_nearest(const void* src, int label_bytes, int C, int D, int H, int W, void* dst, int d, int h, int w,
                         void* stream);
/* Synthetic phantom of one sample on the device (replaces the NIfTI load of dataset.py:74-117 for synthetic
 * runs): label [S^3] (class c+1 inside ellipsoid c = geo[c*6 .. +6) = centre z,y,x, radius z,y,x, first
 * class wins), image [M][S^3] = class_mean[m*(ncls+1) + label] + noise_sd[m] * N (|N| if abs_noise[m]),
 * N standard normal from the SplitMix64 counter stream keys[m] (host array arguments). */
int mmseg_phantom(int S, int ncls, const double* geo, int M, const float* class_mean, const float* noise_sd,
                  const int* abs_noise, const unsigned long long* keys, void* label, int label_bytes, float* image,
                  void* stream);

/* ------------------------------------------------ sliding-window inference */
/* MONAI sliding_window_inference (constant blending) as called by Trainer._sliding_window_inference
 * (trainer.py:370-395).  win: device int[4*nw] = (n, z0, y0, x0) per window in the volume's frame
 * (starts may be negative / past the end: zero padding).  gather: windows [nw][C][r0][r1][r2] of the
 * NCDHW fp32 volume; accum: out[n] += one window's logits [C][r0][r1][r2] (call per window, in order);
 * norm: out /= cz[z] * cy[y] * cx[x] (the per-axis window coverage). */
int mmseg_window_gather(const float* vol, int N, int C, int D, int H, int W, const int* win, int nw, int r0, int r1,
                        int r2, float* out, void* stream);
int mmseg_window_accum(const float* logits, int N, int C, int D, int H, int W, int n, int z0, int y0, int x0, int r0,
                       int r1, int r2, float* out, void* stream);
int mmseg_window_norm(float* out, int N, int C, int D, int H, int W, const float* cz, const float* cy, const float* cx,
                      void* stream);

/* ------------------------------------------------- head, loss, metric */
/* NCDHW fp32 volume channels [c0, c0+cnt) -> NDHWC 8-channel engine layout
 * (batch["image"] as consumed by the first Conv3d, unet.py:181 / dual_encoder.py:133). */
int mmseg_pack_input(const float* x, int Ctot, int c0, int cnt, int N, long long V, void* out, int dtype,
                     void* stream);
/* Same channels packed without padding, (n*V + v)*cnt + c: the stem's input (mmseg_stem_* with ldx = cnt)
 * reads 2*cnt bytes per voxel instead of 16. */
int mmseg_pack_input_compact(const float* x, int Ctot, int c0, int cnt, int N, long long V, void* out, int dtype,
                             void* stream);
/* Dropout3d scale + 1x1 out_conv -> NCDHW fp32 logits (unet.py:195-196). */
int mmseg_head_fwd(const void* x, int ldx, int Cin, const float* W, const float* b, const float* dscale, int C, int N,
                   long long V, float* logits, int dtype, void* stream);
long long mmseg_head_ws_floats(int C, int Cin, int N, long long V);
int mmseg_head_bwd(const void* x, int ldx, int Cin, const float* W, const float* dscale, int C, int N, long long V,
                   const float* dlogits, void* dx, int lddx, float* gW, float* gb, float* ws, int accumulate, int dtype,
                   void* stream);
/* mmseg_head_bwd writing zcols (Cin <= zcols <= lddx, a multiple of 8) channels per dx row: zeros past Cin, so the
 * rows of a dx that owns its padding are written whole (the engine's Act.wcols). */
int mmseg_head_bwd_zw(const void* x, int ldx, int Cin, const float* W, const float* dscale, int C, int N, long long V,
                      const float* dlogits, void* dx, int lddx, int zcols, float* gW, float* gb, float* ws,
                      int accumulate, int dtype, void* stream);
/* Fused softmax + Dice/Tversky + CE statistics and loss (losses.py:39-80, 160-185,
 * 216-228).  type 0: dice_w*Dice + ce_w*CE ; type 1: dice_w*Tversky + ce_w*CE ; type 2: FocalLoss
 * (losses.py:83-125: mean of (1 - exp(-ce_i))^gamma * ce_i with ce_i the class-weighted voxel CE; gamma is
 * passed as alpha, dice_w = 0, ce_w = 1). */
long long mmseg_loss_ws_floats(int N, int C, long long V);
int mmseg_loss_fwd(const float* logits, const void* labels, int label_bytes, int N, int C, long long V, int type,
                   float dice_w, float ce_w, float smooth, float alpha, float beta, int include_bg,
                   const float* class_w, float* loss_out, float* ws, void* stream);
int mmseg_loss_bwd(const float* logits, const void* labels, int label_bytes, int N, int C, long long V, int type,
                   float dice_w, float ce_w, float smooth, float alpha, float beta, int include_bg,
                   const float* class_w, const float* gout, float gconst, float* dlogits, const float* ws,
                   void* stream);
/* Fused training head + loss (the Trainer's fast path, trainer.py:238-243 in one pass each way):
 * forward = head 1x1 conv (+ Dropout3d scale) + mmseg_loss_fwd's statistics without writing the logits;
 * backward = dlogits + the head's data and weight gradient without writing dlogits (logits recomputed with
 * the forward's operation order).  ws: mmseg_loss_ws_floats(N, C, V) floats, same layout (the count of
 * out-of-range labels is its last float); wpart: mmseg_head_loss_wpart_floats() floats.
 * mmseg_head_loss_ok: 1 when (C, Cin, ldx, dtype) has a kernel (2 <= C <= 8, Cin 8, 16 or 32).
 * nmean / nrstd (optional, [N][Cin]): x is the PRE-norm input of the last decoder block's InstanceNorm + ReLU,
 * applied on load exactly as mmseg_instnorm_relu_fwd would (relu((x - mean) * rstd) rounded to the storage
 * type), so that block's output is never written. */
int mmseg_head_loss_ok(int C, int Cin, int ldx, int dtype);
long long mmseg_head_loss_wpart_floats(int C, int Cin, int N, long long V);
int mmseg_head_loss_fwd(const void* x, int ldx, int Cin, const float* nmean, const float* nrstd, const float* W,
                        const float* b, const float* dscale, int C,
                        int N, long long V, const void* labels, int label_bytes, int type, float dice_w, float ce_w,
                        float smooth, float alpha, float beta, int include_bg, const float* class_w, float* loss_out,
                        float* ws, int dtype, void* stream);
int mmseg_head_loss_bwd(const void* x, int ldx, int Cin, const float* nmean, const float* nrstd, const float* W,
                        const float* b, const float* dscale, int C,
                        int N, long long V, const void* labels, int label_bytes, int type, float dice_w, float ce_w,
                        float smooth, float alpha, float beta, int include_bg, const float* class_w, const float* gout,
                        float gconst, const float* ws, void* dx, int lddx, float* gW, float* gb, float* wpart,
                        int accumulate, int dtype, void* stream);
/* mmseg_head_loss_bwd that also emits the InstanceNorm-backward partial sums of the block feeding the head
 * (inpart: [N][mmseg_head_loss_in_chunks()][Cin][2], the layout mmseg_instnorm_bwd_part reads): sums of
 * g = dx [h > 0] and g h per chunk, with h the head's input feature (the normalised, ReLU'd value) and dx the
 * stored data gradient.  Cin == 32 only (mmseg_head_loss_in_chunks() returns 0 otherwise), dx required, dscale
 * (Dropout3d) null. */
int mmseg_head_loss_in_chunks(int C, int Cin, long long V);
int mmseg_head_loss_bwd_in(const void* x, int ldx, int Cin, const float* nmean, const float* nrstd, const float* W,
                           const float* b, const float* dscale, int C,
                           int N, long long V, const void* labels, int label_bytes, int type, float dice_w, float ce_w,
                           float smooth, float alpha, float beta, int include_bg, const float* class_w,
                           const float* gout, float gconst, const float* ws, void* dx, int lddx, float* gW, float* gb,
                           float* wpart, float* inpart, int accumulate, int dtype, void* stream);
/* argmax + per-class intersection / pred / target counts (trainer.py:290-291, metrics.py:42-67). */
int mmseg_dice_counts(const float* logits, const void* labels, int label_bytes, int N, int C, long long V,
                      unsigned long long* counts, void* pred_out, void* stream);
/* counts from class-index masks (DiceMetric.update(pred, target), metrics.py:42-67). */
int mmseg_dice_counts_idx(const void* pred, int pred_bytes, const void* labels, int label_bytes, long long total, int C,
                          unsigned long long* counts, void* stream);
/* AdamW step over flat fp32 buffers (torch.optim.AdamW op order, trainer.py:115-117).
 * skip (nullable): one device float, the step's count of out-of-range labels (mmseg_loss_fwd's last workspace
 * float, summed over the ranks under DP); when it is non-zero the kernel leaves p, m and v untouched, so a batch
 * the trainer raises on (the reference raises in F.one_hot before its optimizer step) never updates the model. */
int mmseg_adamw(float* p, const float* g, float* m, float* v, long long n, float lr, float beta1, float beta2,
                float eps, float wd, int step, const float* skip, void* stream);
/* The same step with its hyper-parameters read from device memory (8 floats), so one launch can be captured
 * in a HIP graph and replayed every step: mmseg_adamw_hyper (host only, no device work) fills the 8 floats for
 * (lr, betas, eps, wd, step) exactly as mmseg_adamw derives them; the caller copies them to the device
 * buffer before each replay. */
int mmseg_adamw_hyper(float lr, float beta1, float beta2, float eps, float wd, int step, float* hyper);
int mmseg_adamw_dev(float* p, const float* g, float* m, float* v, long long n, const float* hyper, const float* skip,
                    void* stream);
/* mmseg_adamw_dev fused with the weight packs (a captured training step's optimizer launch): the same update of
 * the whole arena, and every packed weight's new value also written into its operand images exactly as
 * mmseg_pack_conv3_batched / mmseg_pack_weights_batched write them from the updated weights, so the next forward
 * skips its pack (mmseg_adamw_pack: hyper-parameters by value, as mmseg_adamw).  descs: device table of n descriptors (mmseg_adamw_pack_desc_bytes() each, sorted by first
 * block; built by engine/layers.py Packer.adam_table) covering every arena element exactly once -- 3^3 conv tiles,
 * 1x1 / transposed-conv tiles and plain ranges -- nblocks blocks in all.  p, g, m, v 16-B aligned. */
int mmseg_adamw_pack_desc_bytes(void);
int mmseg_adamw_pack(float* p, const float* g, float* m, float* v, const void* descs, int n, int nblocks, float lr,
                     float beta1, float beta2, float eps, float wd, int step, const float* skip, int dtype,
                     void* stream);
int mmseg_adamw_pack_dev(float* p, const float* g, float* m, float* v, const void* descs, int n, int nblocks,
                         const float* hyper, const float* skip, int dtype, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MMSEG_HIP_H */
