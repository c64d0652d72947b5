/*
 * scdhip.h -- C-ABI of libscdhip.so, the MI355X (gfx950 / CDNA4) kernels behind the
 * scd-resnet training hot path (CenterNet/CornerNet on a ResNet backbone, 512x512 SCD
 * tiles).  Plain C: raw device pointers, sizes and a hipStream_t passed as void*.
 *
 * Conventions
 *   - every entry point returns 0 on success, otherwise a hipError_t code (or SCD_ERR_*);
 *   - no entry point allocates, synchronises or keeps state: work buffers are caller-owned
 *     and sized with the *_workspace helpers; all work is enqueued on `stream`;
 *   - activations are NHWC (channels innermost) in `dtype` (SCD_DT_F32 parity mode,
 *     SCD_DT_BF16 performance mode); weights/grads/BN parameters are fp32 in the
 *     reference (PyTorch) layout so state_dicts interchange; statistics are fp64.
 *
 * Each declaration names the reference interface it replaces (path:line in
 * yang-z-03/scd-resnet @ 2024-10-22).  The reference binds these ops through
 * torch.nn modules (cuDNN/ATen) and, for corner pooling, through pybind11 modules
 * (models/backbones/cornerPooling/source/topPool.cpp:76-85 and siblings); the ctypes binding that
 * replaces both lives in scd-resnet_amd/scdhip/lib.py, see INTEGRATION.md.
 */
#ifndef SCDHIP_H
#define SCDHIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SCD_DT_F32 0
#define SCD_DT_BF16 1
#define SCD_DT_F16 2           /* fp16 operands / activations (v_mfma_f32_16x16x32_f16), fp32 accumulation */

#define SCD_ERR_ARG 9001       /* invalid argument / unsupported shape */

#define SCD_MAX_TAPS 16
#define SCD_MAX_PHASES 4
#define SCD_STAT_REPLICAS 64   /* fp64 statistics buffers are [SCD_STAT_REPLICAS][2][C]; the consumer
                                  (finalize / collapse) re-zeroes what it read, so buffers persist */

/* One sub-pixel phase of a gather-GEMM (see DESIGN.md "Implicit GEMM").  For output
 * pixel (n, qh, qw) of the phase grid, the GEMM row gathers input pixel
 * (n, in_stride*qh + dh[t], in_stride*qw + dw[t]) for tap t and writes output pixel
 * (n, out_stride*qh + rho_h, out_stride*qw + rho_w); tap t uses weight tap wt[t]. */
typedef struct scd_gemm_phase {
    int Qh, Qw, rho_h, rho_w, ntaps;
    int dh[SCD_MAX_TAPS], dw[SCD_MAX_TAPS], wt[SCD_MAX_TAPS];
} scd_gemm_phase;

/* Implicit-GEMM convolution on MFMA (bf16 16x16x32 / f32 16x16x4), NHWC.
 * y[pix, co] = sum_{t,ci} x[gather(pix,t), ci] * w[co, wt(t), ci]  (+bias, relu, +=y)
 * Covers Conv2d forward, Conv2d dgrad (phase-decomposed for stride 2),
 * ConvTranspose2d forward (4 phases) and ConvTranspose2d dgrad.
 * Optionally accumulates per-channel sum/sumsq (fp64, [64][2][Co]) for training BN.
 * Replaces: torch.nn.Conv2d in residuals.py:91,94,211,259-263 (BasicBlock/Bottleneck/stem/
 * downsample), ConvTranspose2d residuals.py:298-307, head convs centerNetOffset.py:106-110,
 * and their autograd input-gradients. */
int scd_conv_gemm(int dtype, const void* x, const void* w, void* y, const float* bias, double* stats,
                  int N, int Hi, int Wi, int Ci, int Ho, int Wo, int Co, int in_stride, int out_stride,
                  int wrow, int relu, int accumulate, int nphase, const scd_gemm_phase* phases,
                  void* stream);

/* scd_conv_gemm (no bias / ReLU / accumulate) whose output y is the gradient dout of a following BN+ReLU
 * layer (pre-BN activation bn_y, same NHWC shape as y): the GEMM epilogue also accumulates that layer's
 * backward sums -- bn_stats[rep][0][c] += sum dz, [rep][1][c] += sum dz*(bn_y-mean)*invstd with
 * dz = y (as stored) where bn_y*relu_scale + relu_shift > 0 -- i.e. what scd_bn_bwd_reduce(y, NULL, bn_y,
 * relu_scale, relu_shift, ...) adds, without re-reading y (ping-pong bf16 GEMM; other shapes run the GEMM and
 * then scd_bn_bwd_reduce).  Replaces the cuDNN input-gradient + BatchNorm2d backward pair of
 * residuals.py:298-307 / centerNetOffset.py:106-110 followed by residuals.py:306. */
/* Input gradient of a 3x3 / stride 2 / pad 1 Conv2d (replaces autograd's cuDNN backward-data of a stride-2 conv,
 * residuals.py:99-103) as ONE forward GEMM: dy (N, Hq, Wq, Cg) gathered at the 2x2 taps (dq, dp) in {0,1}^2, against
 * w3 = pack mode 3 of the (Cg, Cin, 3, 3) weight (4 Cin rows: the four sub-pixel phases, 4 Cg columns), the phases
 * stored as pixels of dx (N, 2Hq, 2Wq, Cin) (+= when accumulate).  SCD_ERR_ARG when the ping-pong GEMM kernel does
 * not take the shape (4 Cin not a multiple of 192 / 256, or fewer than 256 tiles): use scd_conv_gemm then. */
int scd_conv_dgrad_s2(int dtype, const void* dy, const void* w3, void* dx, int N, int Hq, int Wq, int Cg, int Cin,
                      int accumulate, void* stream);
int scd_conv_gemm_bnbwd(int dtype, const void* x, const void* w, void* y, int N, int Hi, int Wi, int Ci, int Ho,
                        int Wo, int Co, int in_stride, int out_stride, int wrow, int nphase,
                        const scd_gemm_phase* phases, const void* bn_y, const float* mean, const float* invstd,
                        const float* relu_scale, const float* relu_shift, double* bn_stats, void* stream);
/* Head convolution with the CenterNet tails fused into the epilogue: hid = relu(conv3x3(x, w) + bias)
 * (N,H,W,nh*128) NHWC and, from the same tile, outs[h] (N,od[h],H,W) fp32 = w1[h] . hid_h + b1[h].
 * Replaces the three terminal Sequentials (centerNetOffset.py:106-110) in one launch; w is the
 * packed [nh*128][9][Ci] operand of the concatenated 3x3 weights. */
int scd_conv_gemm_heads(int dtype, const void* x, const void* w, void* hid, const float* bias, int N, int H,
                        int W, int Ci, int nh, const int* od, const float* const* w1, const float* const* b1,
                        float* const* outs, void* stream);
/* As scd_conv_gemm_heads, with hidden channels >= keep_cols (a multiple of 128) stored only at the pixels where
 * keep[n*H*W + p] != 0 (keep = NULL: all): the size / offset heads' hidden activations are read back by their sparse
 * backward at the loss's gathered pixels only (centerNetOffset.py:199-214), so the forward skips 2/3 of the
 * 403 MB hidden store at B = 32.  Outputs outs[h] are complete either way. */
int scd_conv_gemm_heads_keep(int dtype, const void* x, const void* w, void* hid, const float* bias, int N, int H,
                             int W, int Ci, int nh, const int* od, const float* const* w1, const float* const* b1,
                             float* const* outs, const unsigned char* keep, int keep_cols, void* stream);

/* Weight-gradient of the gather-GEMM (split-K over pixels on MFMA, fp32 partial slabs):
 * ws[z, co, t*Ci+ci] = sum_{pix in split z} g[pix, co] * x[gather(pix, t), ci]
 * with gather(pix=(n,oh,ow), t) = (n, in_stride*oh + dh[t], in_stride*ow + dw[t]).
 * Replaces the weight-gradient half of cuDNN convolution_backward for every Conv2d /
 * ConvTranspose2d above. */
size_t scd_conv_wgrad_workspace(int Cg, int T, int Ci, int nsplit);
/* Number of pixel splits the library picks for an M-pixel weight gradient (tile shape of the
 * kernel it will launch, ~4 waves of workgroups, fp32 slabs capped at 256 MB). */
int scd_conv_wgrad_nsplit(int dtype, long M, int Cg, int T, int Ci);
/* the same knowing the output geometry (selects the 64-pixel ping-pong kernel when Wo % 64 == 0) */
int scd_conv_wgrad_nsplit2(int dtype, long M, int Ho, int Wo, int Cg, int T, int Ci);
int scd_conv_wgrad(int dtype, const void* g, const void* x, float* ws, int nsplit,
                   int N, int Ho, int Wo, int Cg, int Hi, int Wi, int Ci, int in_stride,
                   int T, const int* dh, const int* dw, void* stream);
/* dst[(r-r0)*ld_n + ci*ld_c + t*ld_t] (+)= alpha * sum_z ws[z, r, t*Ci+ci]   for r in [r0,r1), ci < cvalid
 * (alpha = 1 / the fp16 loss scale, else 1) */
int scd_wgrad_reduce(const float* ws, int nsplit, int Cg, int T, int Ci, int r0, int r1, int cvalid,
                     long ld_n, long ld_c, long ld_t, float* dst, int accumulate, float alpha, void* stream);
/* The same over 1..4 row slices [r0[s], r1[s]) with their own destinations and strides, in one launch (the three
 * CenterNet heads' 3x3 weights, centerNetOffset.py:106-110, from one fused weight-gradient workspace).  Requires
 * Ci % 4 == 0.  The summation order over the splits is fixed (independent of the launch geometry). */
int scd_wgrad_reduce_rows(const float* ws, int nsplit, int Cg, int T, int Ci, int nslices, const int* r0,
                          const int* r1, const long* ld_n, const long* ld_c, const long* ld_t, float* const* dst,
                          int cvalid, int accumulate, float alpha, void* stream);

/* Pack an fp32 (A, B, T) weight (OIHW / IOHW flattening) into the GEMM operand layout:
 * mode 0: out[row_off + a][t*B + b] = w[a][b][t]; mode 1: out[row_off + b][t*A + a] = w[a][b][t];
 * rows are ldp elements long (zero padded).  mode 2 (tap-major transpose): out[t*B + b][row_off + a] = w[a][b][t],
 * T*B rows of ldp elements of which only [row_off, row_off + A) are written (one slice of a concatenation).
 * mode 3 (T = 9, ldp >= 4A): out[row_off + (2 rh + rw) B + b][(2 dq + dp) A + a] = w[a][b][rh + 1 - 2 dq][rw + 1 - 2 dp]
 * (zero outside the kernel): the operand of scd_conv_dgrad_s2. */
int scd_pack_weight(int dtype, const float* w, void* out, int A, int B, int T, int mode, int ldp,
                    int row_off, void* stream);

/* Zero-extend the innermost dimension: dst[r][c] = c < C ? src[r][c] : 0 (r < rows, c < Cp).  Lets the gather-GEMM
 * run layers narrower than its K-stage (the 16/32-channel `*h` / `*q` plugins, trainer/model/centerOffsetRes10q.py):
 * the input (rows = pixels) and the packed operand (rows = output rows x taps) are padded to the next multiple
 * of 64 (bf16) / 32 (fp32) channels.  C, Cp multiples of 8 (bf16) / 4 (fp32). */
int scd_pad_channels(int dtype, const void* src, long rows, int C, int Cp, void* dst, void* stream);

/* Batched weight packing: all operand layouts of one training step in one launch.  descs (device memory)
 * are sorted by start; descriptor d covers elements [start, start + count) of the concatenated index space:
 * mode 0: out[row_off + a][t*B + b] = w[a][b][t], count = A * ldp (k >= T*B zero-filled);
 * mode 1: out[b][t*a_tot + a_off + a] = w[a][b][t] (a slice of a concatenated operand when a_tot > A),
 * transposed through LDS in tiles of 64 a x max(1, 64/T) b (T <= 64), one 4096-element unit per tile:
 * count = 4096 * ceil(A/64) * ceil(B / max(1, 64/T)); mode 2: out[t*B + b][a_off + a] = w[a][b][t] (ldp = a_tot),
 * count = A * B * T; mode 3 (T = 9, ldp = 4A): out[row_off + (2 rh + rw) B + b][(2 dq + dp) A + a] =
 * w[a][b][rh + 1 - 2 dq][rw + 1 - 2 dp] (zero outside the 3x3 kernel; scd_conv_dgrad_s2's operand), count = 16 A B.
 * Every start (and total) is a multiple of 4096.
 * Replaces one scd_pack_weight launch per conv and direction. */
typedef struct scd_pack_desc {
    const float* w;
    void* out;
    long start;
    int A, B, T, mode, ldp, row_off, a_off, a_tot;
} scd_pack_desc;
int scd_pack_weights_batched(int dtype, const scd_pack_desc* descs, int n, long total, void* stream);

/* Stem im2col: x (N,1,H,W) fp32 -> cols (N,Ho,Wo,Kpad) dtype, taps kh*kw zero-padded to Kpad.
 * Feeds residuals.py:211 (Conv2d(1,64,7,s2,p3)) to the MFMA GEMM as a 1x1 conv. */
int scd_im2col_stem(int dtype, const float* x, void* cols, int N, int H, int W, int Ho, int Wo, int kh,
                    int kw, int stride, int pad, int Kpad, void* stream);

/* Direct stem convolution (bf16): Conv2d(1,64,7,stride 2,pad 3,no bias) of residuals.py:211 with the
 * [pixel][tap] tile built in LDS from the input patch (no column tensor in HBM); wpk = the [64][64] packed
 * weight (pack_weight mode 0, ldp 64); y (N,Ho,Wo,64) NHWC; stats as scd_conv_gemm (may be NULL).
 * Requires Wo % 128 == 0 and Ho % 2 == 0. */
int scd_stem_conv_fwd(int dtype, const float* x, const void* wpk, void* y, double* stats, int N, int H, int W,
                      int Ho, int Wo, void* stream);
/* Its weight gradient: ws[z][co][k] (fp32, nsplit x 64 x 64) = sum over split z's pixels of
 * dy[pix][co] * col[pix][k]; reduce with scd_wgrad_reduce(ws, nsplit, 64, 1, 64, ..., cvalid = 49).
 * coef != NULL fuses the stem BN backward apply: dy is then the masked dz, ybn the BN input, and the
 * operand is bf16(coef[0][c]*dz + coef[1][c]*ybn + coef[2][c]) (scd_bn_bwd_finalize's coefficients).
 * Requires Wo % 64 == 0. */
int scd_stem_conv_wgrad_nsplit(long M);
int scd_stem_conv_wgrad(int dtype, const void* dy, const void* ybn, const float* coef, const float* x, float* ws,
                        int nsplit, int N, int H, int W, int Ho, int Wo, void* stream);
/* Stem backward in one pass (residuals.py:209-216 backward, replacing autograd's MaxPool2d / ReLU / BatchNorm2d /
 * Conv2d backward chain of the stem): from the pooled gradient dout (N,Ho/2,Wo/2,64), its argmax, the pre-BN conv
 * output y (N,Ho,Wo,64) and the input x (N,1,H,W) fp32, accumulates the BN backward sums (sum dz, sum dz*xhat) into
 * stats (fp64 replicas, as scd_stem_pool_bwd_bn) and writes tg = [T1 | G] (2 x 64 x 64 fp32: sum dz col^T and the
 * Gram matrix of the input columns, tap 49 = 1), via ws (scd_stem_bwd_nsplit() x 2 x 64 x 64 floats).
 * scd_stem_bwd_combine then adds dW = alpha (a T1 + b W G + c s) with (a, b, c) = scd_bn_bwd_finalize's coefficients
 * and W = the forward's packed bf16 weights (64 x 64) into dst (64,1,7,7). */
int scd_stem_bwd_nsplit(void);
int scd_stem_bwd_fused(int dtype, const void* dout, const uint8_t* argmax, const void* y, const float* scale,
                       const float* shift, const float* mean, const float* invstd, const float* x, double* stats,
                       float* ws, int nsplit, float* tg, int N, int H, int W, int Ho, int Wo, void* stream);
int scd_stem_bwd_combine(int dtype, const float* tg, const void* wpk, const float* coef, float* dst, int accumulate,
                         float alpha, void* stream);

/* ---- training BatchNorm2d (residuals.py:92,95,212,262,306; momentum 0.1, eps 1e-5) ---- */
/* sum replicas [nrep][2][C] -> [2][C] in place (replica 0); used before a SyncBN all-reduce */
int scd_stats_collapse(double* stats, int nrep, int C, void* stream);
/* out[0 .. 2C) = the replica sum of stats, every replica zeroed: two BN layers' sums collapsed side by side into one
 * staging buffer go through ONE SyncBN all-reduce (networkFactory.py:128-133), then finalize with nrep = 1 */
int scd_stats_collapse_to(double* stats, int nrep, int C, double* out, void* stream);
/* mean/var from stats (count rows), running-stat update (unbiased var), scale/shift for apply;
 * stats == NULL: eval mode, normalise with the running statistics (no update) */
int scd_bn_finalize(double* stats, int nrep, int C, double count, const float* gamma,
                    const float* beta, float* running_mean, float* running_var, int64_t* num_batches,
                    float momentum, float eps, float* mean, float* invstd, float* scale, float* shift,
                    void* stream);
/* Several layers' finalizes in ONE launch (a block's bn1 and downsample BN, whose statistics are complete together;
 * residuals.py:99-120): layers[0 .. n) as scd_bn_finalize's arguments, n <= SCD_BN_FIN_MAX (host array). */
#define SCD_BN_FIN_MAX 4
typedef struct scd_bn_fin_args {
    double* stats;             /* [nrep][2][C] fp64 sums, zeroed after reading (NULL: eval mode) */
    int nrep, C;
    double count;
    const float* gamma;
    const float* beta;
    float* running_mean;
    float* running_var;
    int64_t* num_batches;
    float momentum, eps;
    float* mean;
    float* invstd;
    float* scale;
    float* shift;
} scd_bn_fin_args;
int scd_bn_finalize_n(const scd_bn_fin_args* layers, int n, void* stream);
/* out = act(y*scale + shift + R), R = 0 | res | res*rscale + rshift */
int scd_bn_apply(int dtype, const void* y, void* out, int C, long total, const float* scale,
                 const float* shift, const void* res, const float* rscale, const float* rshift,
                 int relu, void* stream);
/* dz = dout * relu'(.) ; stats += [sum dz, sum dz*(y-mean)*invstd].  relu' from the stored activation
 * (mask > 0) or, for a plain BN+ReLU (mask == NULL, relu_scale != NULL), from the forward's own
 * y*relu_scale + relu_shift > 0 (no activation read); both NULL: no ReLU. */
int scd_bn_bwd_reduce(int dtype, const void* dout, const void* mask, const void* y, const float* relu_scale,
                      const float* relu_shift, const float* mean, const float* invstd, int C, long total,
                      double* stats, void* stream);
/* dgamma (+)= gscale * sum dz*xhat, dbeta (+)= gscale * sum dz; coef[3][C] for dy = a*dz + b*y + c.
 * With SyncBN the sums are global; gscale = 1/world keeps the DDP-averaged dgamma/dbeta equal to the
 * reference's (torch SyncBatchNorm returns the LOCAL weight/bias gradients, DDP then averages them). */
int scd_bn_bwd_finalize(double* stats, int nrep, int C, double count, const float* gamma,
                        const float* mean, const float* invstd, float* dgamma, float* dbeta,
                        float gscale, float* coef, void* stream);
/* ... several layers in ONE launch (the two BN layers behind a residual join, whose sums scd_bn_bwd_reduce2 makes
 * together): layers[0 .. n) as scd_bn_bwd_finalize's arguments, n <= SCD_BN_FIN_MAX (host array) */
typedef struct scd_bn_bwd_fin_args {
    double* stats;
    int nrep, C;
    double count;
    const float* gamma;
    const float* mean;
    const float* invstd;
    float* dgamma;
    float* dbeta;
    float gscale;
    float* coef;
} scd_bn_bwd_fin_args;
int scd_bn_bwd_finalize_n(const scd_bn_bwd_fin_args* layers, int n, void* stream);
/* dy = a*dz + b*y + c (dtype), dz masked as in scd_bn_bwd_reduce; optionally also writes dz */
int scd_bn_bwd_apply(int dtype, const void* dout, const void* mask, const void* y, const float* relu_scale,
                     const float* relu_shift, const float* coef, int C, long total, void* dy, void* dz,
                     void* stream);

/* Two BN layers behind one residual join (BasicBlock bn2 / Bottleneck bn3 + the downsample BN, residuals.py:110-120,
 * 158-165; CornerPool branchMergeBn + shortcutBn, cornerNetCPool.py:117-122): the same gradient dout and ReLU mask
 * (mask > 0, required) for both.  scd_bn_bwd_reduce2 = scd_bn_bwd_reduce for (ya, stats_a) and (yb, stats_b) in one
 * pass; scd_bn_bwd_apply2 = scd_bn_bwd_apply for (ya, coef_a -> dya) and (yb, coef_b -> dyb) in one pass. */
int scd_bn_bwd_reduce2(int dtype, const void* dout, const void* mask, const void* ya, const void* yb,
                       const float* mean_a, const float* invstd_a, const float* mean_b, const float* invstd_b, int C,
                       long total, double* stats_a, double* stats_b, void* stream);
int scd_bn_bwd_apply2(int dtype, const void* dout, const void* mask, const void* ya, const void* yb,
                      const float* coef_a, const float* coef_b, int C, long total, void* dya, void* dyb, void* stream);


/* ---- stem BN-apply + ReLU + MaxPool2d(3,2,1) (residuals.py:212-214) ---- */
/* MaxPool backward + ReLU mask (as scd_stem_pool_bwd) fused with the stem BN backward reduction:
 * also stats[rep][2][C] += [sum dz, sum dz*(y-mean)*invstd] over the rounded dz it writes. */
int scd_stem_pool_bwd_bn(int dtype, const void* dout, const uint8_t* argmax, const void* y, const float* scale,
                         const float* shift, const float* mean, const float* invstd, void* dz, double* stats, int N,
                         int H, int W, int C, int Ho, int Wo, void* stream);
int scd_stem_pool_fwd(int dtype, const void* y, const float* scale, const float* shift, void* out,
                      uint8_t* argmax, int N, int H, int W, int C, int Ho, int Wo, void* stream);
/* dz(N,H,W,C) = relu'(y*scale+shift) * maxpool_bwd(dout) */
int scd_stem_pool_bwd(int dtype, const void* dout, const uint8_t* argmax, const void* y,
                      const float* scale, const float* shift, void* dz, int N, int H, int W, int C,
                      int Ho, int Wo, void* stream);

/* ---- fused CenterNet head tails: ReLU'd hidden (N,HW,nh*Hd) -> per-head 1x1 conv + bias ----
 * Replaces the terminal Conv2d(128, {1,4,2}, 1) at centerNetOffset.py:108-110 (and its
 * autograd).  Head h reads hidden channels [h*Hd, (h+1)*Hd); w1[h] is its fp32 (od[h], Hd)
 * weight, b1[h] its bias; outputs are NCHW fp32 (N, od[h], HW).  nh <= 4, od[h] <= 4. */
int scd_heads_fwd(int dtype, const void* hid, int N, int HW, int nh, int Hd, const int* od,
                  const float* const* w1, const float* const* b1, float* const* outs, void* stream);
/* fused tail backward: dhid = relu'(hid) * (w1^T dout) (dtype) and, in the same pass,
 * acc (fp64, [SCD_STAT_REPLICAS][sum(od)*Hd | sum(od) | nh*Hd]) += [dW1 | db1 | db0] */
size_t scd_heads_bwd_accsize(int nh, int Hd, const int* od);
int scd_heads_bwd(int dtype, const void* hid, int N, int HW, int nh, int Hd, const int* od,
                  const float* const* w1, const float* const* douts, void* dhid, double* acc, void* stream);
/* collapse (and re-zero) acc; (+)= into dw1[h] (od[h],Hd), db1[h] (od[h]), db0[h] (Hd: 3x3 conv bias) */
/* scd_heads_bwd with the head-output gradients first repacked pixel-major into `packed` ([N*HW][nh][4] fp32,
 * caller-allocated, zero padded) and multiplied by dscale (the fp16 loss scale, else 1): one 16-B gradient read per
 * pixel and head instead of od scalar reads. */
int scd_heads_bwd_packed(int dtype, const void* hid, int N, int HW, int nh, int Hd, const int* od,
                         const float* const* w1, const float* const* douts, float dscale, float* packed, void* dhid,
                         double* acc, void* stream);
int scd_heads_bwd_weight_finalize(double* acc, int nh, int Hd, const int* od, float* const* dw1,
                                  float* const* db1, float* const* db0, int accumulate, float alpha, void* stream);
/* The same tail backward over the dense heads [0, nd) only: dhid has row stride nd*Hd (hid keeps nh*Hd), packed
 * is [pixel][nd][4].  scd_heads_bwd_packed == scd_heads_bwd_packed_split with nd = nh. */
int scd_heads_bwd_packed_split(int dtype, const void* hid, int N, int HW, int nh, int Hd, const int* od, int nd,
                               const float* const* w1, const float* const* douts, float dscale, float* packed,
                               void* dhid, double* acc, void* stream);
/* Heads [nd, nh) whose output gradients vanish outside the pixels inds[b][k] (b < N, k < K; HW-local indices): the
 * regression / offset terminals under L1LossMask(gather(out, inds), ..., mask) (centerNetOffset.py:199-214,
 * regression.py:37-44; utility.py:76-85 gather).  Slot s = b*K + k; the first slot naming a pixel is active.
 * scd_heads_sparse_bwd: dhid_s[s][(nh-nd)*Hd] = relu'(hid) * W1^T g (zero rows for inactive slots),
 * xcol[s][t*Cin + ci] = the slot pixel's 3x3 patch of feat (tap-major; zeros outside the image), the
 * heads' dW1/db1/db0 into acc (scd_heads_bwd_weight_finalize), slotmap[pixel] = s, ownermap[q] = min(s*9 + t)
 * over the (slot, tap) pairs reaching q.  scd_heads_sparse_fixup: dx[q] += sum over taps t of
 * cols[slot(q - d_t)][t*Cin + ci] (cols = dhid_s x W0^T, the 3x3 conv's weight packed tap-major as a [9*Cin][Cs] GEMM
 * operand) at every reached q, with the following BN+ReLU layer's backward sums corrected when bn_y != NULL
 * (scd_conv_gemm_bnbwd's definition); both maps are restored (slotmap = -1, ownermap = INT_MAX: persistent
 * int32[N*H*W] buffers initialised once).  (nh-nd)*Hd <= 256, Cin <= 256. */
int scd_heads_sparse_bwd(int dtype, const void* hid, const void* feat, int N, int H, int W, int Cin, int nh, int Hd,
                         const int* od, int nd, const float* const* w1, const float* const* douts, float dscale,
                         const long* inds, int K, void* dhid_s, void* xcol, double* acc, int* slotmap, int* ownermap,
                         void* stream);
int scd_heads_sparse_fixup(int dtype, void* dx, const void* cols, int N, int H, int W, int Cin, const long* inds, int K,
                           int* slotmap, int* ownermap, const void* bn_y, const float* mean, const float* invstd,
                           const float* relu_scale, const float* relu_shift, double* bn_stats, void* stream);

/* ---- losses (focal.py:25-53, regression.py:37-44, centerNetOffset.py:182-217) ---- */
/* per element: g = d/dlogit [pos: log(p)(1-p)^2 | neg: log(1-p) p^2 (1-gt)^4] with
 * p = clamp(sigmoid(x),1e-4,1-1e-4); acc[0..2] (fp64, replicated [64][4]) += posL, negL, npos */
int scd_focal_fwd(const float* logits, const float* gt, long n, float* g, double* acc, void* stream);
/* masked L1 on gathered NCHW features: acc[0] += sum |f-t|, acc[1] += sum mask; g = sign(f-t) scattered */
int scd_l1_gather_fwd(const float* feat, int N, int C, int HW, const int64_t* inds, const uint8_t* mask,
                      const float* target, int K, int tstride, int toff, float* g, double* acc, void* stream);
/* out[0..] = loss terms; factors for backward.  See centerNetOffset.py:213-217.  Re-zeroes focal_acc and
 * l1_acc after reading them (persistent accumulators: no memset before the next loss). */
int scd_centernet_loss_finalize(double* focal_acc, int nfocal, double* l1_acc, int nl1,
                                const float* l1_weights, float* out, float* factors, void* stream);
/* CenterNetLoss (centerNetOffset.py:182-217) in two launches: the focal loss + gradient on the heatmap logits (as
 * scd_focal_fwd) with the zero fill of the size / offset gradient buffer (g_off must follow g_regr in memory), then
 * one workgroup for both masked L1 terms (regr: target channels toff_r.., off: toff_o.., as scd_l1_gather_fwd) and
 * the finalize (as scd_centernet_loss_finalize with nfocal = 1, nl1 = 2: out = [loss, focal, size, offset],
 * factors = the three backward scales; focal_acc re-zeroed).  scd_centernet_loss_bwd_scale: g_heat *= factors[0]*go;
 * g_regr / g_off (zero except at the gathered pixels) scaled by factors[1] / factors[2]*go at those pixels only,
 * each once. */
int scd_centernet_loss_fwd(const float* heat, const float* gt, long n_heat, const float* regr, int Cr, const float* off,
                           int Co, int N, int HW, const int64_t* inds, const uint8_t* mask, const float* target, int K,
                           int tstride, int toff_r, int toff_o, const float* l1_weights, float* g_heat, float* g_regr,
                           float* g_off, double* focal_acc, float* out, float* factors, void* stream);
int scd_centernet_loss_bwd_scale(float* g_heat, long n_heat, int N, int HW, const int64_t* inds, int K, float* g_regr,
                                 int Cr, float* g_off, int Co, const float* factors, const float* go, void* stream);

/* Keep map for scd_conv_gemm_heads_keep from the loss targets' gather indices inds (N,K) int64 (the `inds` target of
 * CenterNetLoss, centerNetOffset.py:199-214): keep[n*HW + inds[n][k]] = 1 for every slot, after clearing the pixels
 * the previous call set (prev: nprev >= N*K int64, -1-filled on first use, updated in place; keep zero-filled on
 * first use).  One workgroup. */
int scd_heads_keep_map(const int64_t* inds, int N, int K, int HW, int64_t* prev, int nprev, uint8_t* keep, void* stream);

/* g[i] *= factors[idx] * go[0]  (in place) */
int scd_scale_by_device(float* g, long n, const float* factors, int idx, const float* go, void* stream);

/* CenterNet training targets on the GPU (datasets/scds/scdx16p100.py:514-531, :575-591,
 * datasets/utility.py:11-16, evaluations/intersection.py:46-63): locs (B,K,8) fp32 object rows
 * [ctx, cty, offx, offy, majx, majy, minl, halo], counts (B) int32 objects per tile (<= K <= 64) ->
 * heat (B,1,H,H) fp32 (Gaussian splats in object order, each added in float64 and clipped at 1),
 * mask (B,K) u8, regr (B,K,6) fp32 = locs[..., 2:8], inds (B,K) int64 = floor(cty)*H + floor(ctx)
 * (0 where the centre is outside the map). threshold = the IoU threshold of the radius rule (0.5). */
int scd_render_center_targets(const float* locs, const int* counts, int B, int K, int H, float threshold,
                              float* heat, uint8_t* mask, float* regr, int64_t* inds, void* stream);
/* SCD tile augmentation (datasets/scds/scdx16p100.py:416-441, datasets/argumentations.py:38-64):
 * out[b] = (flip(in[b]) - mean) / sqrt(var) * jitter[b] + noise * noise_sv, mean/var over the flipped tile (fp64
 * sums).  flips (B,2) u8 device [x (dim 2), y (dim 1)], nullable; jitter (B) device factors (1 + 0.05 g), nullable;
 * noise (B,H,W) device N(0,1) draws, or NULL for the counter-based generator keyed by seed; noise_sv 0 = no noise
 * (the validation set's normalize alone).  W % 4 == 0, in != out.  workspace: scd_augment_workspace(B) bytes. */
size_t scd_augment_workspace(int B);
int scd_augment_tiles(const float* in, float* out, int B, int H, int W, const uint8_t* flips, const float* jitter,
                      const float* noise, float noise_sv, unsigned long long seed, void* workspace, void* stream);
/* ---- whole-slide tiled inference (test.py:19-135) ----
 * scd_slide_tiles: RGB slide (H,W,C>=3) u8 on the device -> out (clipH*clipV, 1, tile, tile) fp32 clips, x-major,
 * grey = round(0.1140 c0 + 0.5870 c1 + 0.2989 c2) (float64), torch-'reflect' padding by padLR / padTB, the
 * reference's opencv column fix-up when fix != 0 (needs a padded width >= 3200), each clip normalised in float64.
 * workspace: scd_slide_workspace(clipH*clipV) bytes.
 * scd_slide_detections: decoded (10, T, K) fp32 Wrapper stack (trainer/wrappers/centerOffsetResidual.py:10-23)
 * -> the detections with score > thr in tile-then-rank order: xy (n,2) int32 slide pixels, ratio (n) float64,
 * *count = n (device); xy / ratio sized T*K. */
size_t scd_slide_workspace(int ntiles);
int scd_slide_tiles(const uint8_t* rgb, int H, int W, int C, int tile, int stride, int clipH, int clipV, int padLR,
                    int padTB, int fix, float* out, void* workspace, void* stream);
int scd_slide_detections(const float* decoded, int T, int K, int stride, int padLR, int padTB, int clipV, float thr,
                         int* xy, double* ratio, int* count, void* stream);
/* ---- decode (centerNetOffset.py:219-251, utility.py:87-118) ---- */
size_t scd_decode_workspace(int N, int HW);
int scd_decode_topk(const float* heat, int N, int H, int W, int K, const float* offset, int od_off,
                    const float* regr, int od_regr, float* scores, int64_t* inds, int64_t* ys, int64_t* xs,
                    float* off_out, float* regr_out, void* workspace, void* stream);

/* ---- validation metrics (models/centerNetOffset.py:253-354, evaluations/detection.py:11-230,
 * trainer/model/centerOffsetRes10.py:18-106) ----
 * Decoded detections (scores/cty/ctx (N,K), offset (N,K,2), regr (N,K,4)) against ground truth (gt_regr (N,L,6);
 * gt_loc = heat indices (N,L) int64 when loc_mode 0, or locs rows (N,L,loc_w) fp32 [x, y, ...] when loc_mode 1),
 * H = heatmap width, thr = the score threshold of validMask (0.3).  K <= 256, L <= 64.
 * Nine value streams, each the masked_select of the reference in (n,k,l) order:
 *   0 IoUConfidence iou, 1 IoUConfidence score, 2 Orthogonity, 3 IoU centre/centre, 4 IoU centre/offset (iouoffsetwo),
 *   5 IoU offset/offset, 6-8 MAE majL/minL/halo.   Masks: streams 0,1 -> mask 0; 2,6,7,8 -> mask 1; 3 -> 2; 4 -> 3;
 *   5 -> 4.  scd_ceval_count writes counts (N,5) int32; scd_ceval_emit writes every stream at its exact offset
 *   (streams[9] device pointers, sized by the column sums of counts). */
int scd_ceval_count(const float* scores, const int64_t* cty, const int64_t* ctx, const float* offset, const float* regr,
                    const float* gt_regr, const void* gt_loc, int loc_mode, int loc_w, int N, int K, int L, int H,
                    float thr, int* counts, void* stream);
int scd_ceval_emit(const float* scores, const int64_t* cty, const int64_t* ctx, const float* offset, const float* regr,
                   const float* gt_regr, const void* gt_loc, int loc_mode, int loc_w, int N, int K, int L, int H,
                   float thr, const int* counts, float* const* streams, void* stream);
/* expression(): out[0..8] = fp64 means of the nine streams (stream 2 over its non-NaN values), out[9+t] = the
 * reference's interpolated AP (averagePrecisionPlots + averagePrecisionAll) of stream 0 ranked by stream 1 at
 * IoU threshold thr[t] (device array), objects = max(objnum, lens[0]).  Ranking: score descending, ties by
 * descending pair index.  streams/lens are HOST arrays of 9 (device pointers / lengths). */
size_t scd_ceval_summary_workspace(long n);
int scd_ceval_summary(const float* const* streams, const long* lens, long objnum, const float* thr, int nthr,
                      double* out, void* workspace, void* stream);

/* ---- Adam (torch.optim.Adam defaults, networkFactory.py:79-82) over a flat fp32 buffer ---- */
int scd_adam_step(float* p, const float* g, float* m, float* v, long n, float lr, float beta1, float beta2,
                  float eps, float bc1, float bc2, float gscale, void* stream);
/* Same update with the step state in device memory: hyper = {lr, step} (fp64, step advanced by 1 on the stream
 * before the update), so a captured training-step graph (scdhip/graph.py) replays with the live learning rate and
 * bias corrections (networkFactory.py:228-234, :273-276).  skip (optional device word; the peer-memory SyncBN error
 * word, scdhip/peer.py): non-zero = the gradients were formed from unreduced statistics -- nothing changes (step count,
 * parameters, moments). */
int scd_adam_step_dev(float* p, const float* g, float* m, float* v, long n, double* hyper, float beta1, float beta2,
                      float eps, float gscale, const unsigned long long* skip, void* stream);
/* ---- SGD (torch.optim.SGD, networkFactory.py:84-89: momentum 0.9, weight_decay 1e-4) over a flat fp32 buffer ----
 * hyper = {lr, step, initialised, scratch} (fp64, 4 values): step advanced on the stream as for scd_adam_step_dev;
 * the momentum buffer `buf` is initialised to this step's d = g*gscale + weight_decay*p (as torch clones it when the
 * parameter has no momentum_buffer yet) when hyper[2] == 0, and hyper[2] is set to 1 -- a per-buffer flag, so a
 * buffer rebuilt or reset mid-training starts like torch's, whatever the step.  buf may be NULL when momentum == 0. */
int scd_sgd_step_dev(float* p, const float* g, float* buf, long n, double* hyper, float momentum, float dampening,
                     float weight_decay, int nesterov, float gscale,
                     const unsigned long long* skip, void* stream);

/* ---- corner pooling (cornerPooling/source/{top,bottom,left,right}Pool.cpp) ----
 * dir: 0 top (max over k>=h), 1 bottom (k<=h), 2 left (k>=w), 3 right (k<=w); NHWC dtype.
 * Backward routes grad to the running argmax, ties keep the first-scanned index
 * (strict '>' update, topPool.cpp:61-65), each run summed in scan order as the reference's scatter_add loop
 * (topPool.cpp:56-70): fp32 results are bit-identical to the reference backward's. */
int scd_cpool_fwd(int dtype, int dir, const void* x, const void* addend, void* y, int N, int H, int W, int C,
                  void* stream);                     /* y = pool(x) (+ addend, nullable: the CornerPool branch sum) */
int scd_cpool_bwd(int dtype, int dir, const void* x, const void* dy, void* dx, int N, int H, int W, int C,
                  void* stream);

/* library self-description (for the loader / tests) */
/* ---- the reference's functional helpers, for user code that calls them directly (fp32, device pointers) ----
 * scd_nms: out = x * (x == max over its k x k window, -inf padded), k odd -- utility.py:87-92 nonMaximumSuppression.
 * scd_topk: per row of B x n scores, the K (<= 1024) largest (ties by ascending index) with the reference's split of
 * the flat index into category = i / HW, index = i % HW, y = index / W, x = index % W -- utility.py:106-118.
 * scd_focal_prob_fwd: focal.py:25-53 on probabilities: g = d(posL + negL)/dp per element, acc[rep][4] += {posL, negL,
 * #pos}; scd_centernet_loss_finalize(acc, 1, NULL, 0, ...) forms the loss and the normaliser factor.
 * scd_masked_l1_fwd: regression.py:28-44 on (rows, C) gathered values: acc[0..1] += {sum of |d| (smooth: smooth-L1,
 * beta 1) over masked rows, #masked rows}, g = d/d(r) of that sum (0 on unmasked rows). */
int scd_nms(const float* x, long planes, int H, int W, int k, float* out, void* stream);
int scd_topk(const float* scores, int B, long n, int K, int HW, int W, float* out_scores, int64_t* inds, int* cats,
             float* ys, float* xs, void* stream);
int scd_focal_prob_fwd(const float* p, const float* gt, long n, float* g, double* acc, void* stream);
int scd_masked_l1_fwd(const float* r, const float* t, const uint8_t* mask, long rows, int C, int smooth, float* g,
                      double* acc, void* stream);

/* ---- SyncBN over peer memory (networkFactory.py:128-133: SyncBatchNorm on multi-GPU runs) ----
 * A one-shot all-reduce of <= cap doubles for R <= 8 ranks without a collective library: every rank allocates a
 * fine-grained mailbox (scd_peer_alloc, scd_peer_mailbox_bytes(R, cap) bytes, zeroed), exports it
 * (scd_peer_ipc_handle: 64 bytes) and maps the others' (scd_peer_ipc_open); scd_peer_allreduce_f64 then writes
 * `data` into every mailbox, flags it with `epoch` (1, 2, 3, ... one per call, the same on every rank), waits for
 * all flags and leaves the rank-ordered sum in `data` (identical bits on every rank).  boxes[r] = rank r's mailbox
 * as mapped in this process.  A late peer is waited for up to timeout_ms (a sleeping one-wave poll); if its flag is
 * still missing then, *err (device, zero-initialised) receives the failing epoch and data is left unreduced.  The
 * error is sticky: a call that finds *err != 0 does nothing.  The host reads *err once per step (scdhip/peer.py).
 * The allocation entry points are the only ones in this library that allocate. */
size_t scd_peer_mailbox_bytes(int R, int cap);
int scd_peer_alloc(size_t bytes, void** ptr);
int scd_peer_free(void* ptr);
int scd_peer_ipc_handle(void* ptr, void* handle64);
int scd_peer_ipc_open(const void* handle64, void** ptr);
int scd_peer_ipc_close(void* ptr);
int scd_peer_allreduce_f64(double* data, int n, int rank, int R, void* const* boxes, int cap, unsigned long long epoch,
                           unsigned long long* err, unsigned timeout_ms, void* stream);


/* ---- HIP events for live kernel timing (bench.py roofline; scdhip.ops.LaunchTimer) ----
 * scd_event_record stamps the event on `stream`; while the stream is being captured into a graph the record is an
 * external event node (hipEventRecordExternal), re-stamped by every replay.  scd_event_elapsed_ms waits for `end`. */
int scd_event_create(void** ev);
int scd_event_destroy(void* ev);
int scd_event_record(void* ev, void* stream);
int scd_event_elapsed_ms(void* start, void* end, float* ms);

/* ---- calibration (diagnostics; SURVEY.md §8(d) C2: the achievable MFMA peak on the box) ----
 * scd_calib_mfma_peak: grid workgroups of 4 waves, each running `iters` x 16 v_mfma_f32_16x16x32_bf16 on random bf16
 * fragments read from `src` (>= 256 x 8 x 64 x 16 bytes); out: grid x 256 floats (keeps the accumulators live);
 * stamps (optional): [grid x 4 waves][4] = {s_memtime at loop start, at loop end, s_memrealtime at start, at end}.
 * scd_calib_set_stamps: the [workgroup][4] buffer the GEMM kernels of a stamped diagnostic build write their main-loop
 * stamps to (scd_calib_stamped_build() == 1); the product build never writes it. */
int scd_calib_mfma_peak(const void* src, int grid, int iters, float* out, unsigned long long* stamps, void* stream);
int scd_calib_set_stamps(unsigned long long* stamps);
int scd_calib_stamped_build(void);

/* library identity: "libscdhip <abi> gfx950 <hash of the sources built>" */
const char* scd_version(void);

#ifdef __cplusplus
}
#endif
#endif
