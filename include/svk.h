/*
 * svk.h — C ABI of the MI355X (gfx950) kernel library behind the build's
 * `models.*` drop-in surface for the surgical-phase hot path.
 *
 * The reference (THao712/Deep-Learning-for-Surgical-Video-Analysis) exposes no
 * FFI: its boundary is the Python module/class surface.  Each
 * entry point below replaces the PyTorch op(s) the reference calls at the cited
 * file:line; the Python host (svk/_lib.py, ctypes) binds exactly these symbols.
 *
 * Conventions
 *   - Caller owns all memory (device pointers; the library never allocates).
 *   - Stream-ordered and asynchronous: `stream` is a hipStream_t (NULL = default
 *     stream); no host synchronisation inside any call.
 *   - Return 0 on success, negative SVK_E* on error; svk_last_error() gives a
 *     thread-local message.  No exceptions cross the ABI.
 *   - dtype selects the storage/compute type of activations and weights:
 *     SVK_F32 (f32 MFMA, exact f32 products, parity path), SVK_F16 (f16 MFMA, f32
 *     accumulation: the precision of the reference's torch.autocast(float16) regions,
 *     train_evp.py:493/637/760) or SVK_BF16 (bf16 MFMA, f32 accumulation).  Biases, norm
 *     affine terms and depthwise taps are f32; statistics and accumulation are f32 for
 *     every dtype.
 *   - Token layouts are row-major [rows, channels] with an explicit leading
 *     dimension; image/feature maps are NHWC (token n = h*W + w, the reference's
 *     own `flatten(2).transpose(1, 2)` order, mix_transformer_evp.py:212).
 */
#ifndef SVK_H
#define SVK_H

#ifdef __cplusplus
extern "C" {
#endif

enum { SVK_F32 = 0, SVK_BF16 = 1, SVK_F16 = 2 };
enum { SVK_ACT_NONE = 0, SVK_ACT_GELU = 1, SVK_ACT_RELU = 2, SVK_ACT_TANH = 3 };
enum { SVK_OK = 0, SVK_EINVAL = -1, SVK_EUNSUPPORTED = -2, SVK_ELAUNCH = -3 };

const char* svk_version(void);
const char* svk_last_error(void);
/* Kernel instantiation launched last by the calling thread (GEMM / conv family; for profilers). */
const char* svk_last_kernel(void);
/* Tuning knobs for A/B measurements inside one process (no effect on results: every setting selects a
 * complete, parity-tested kernel variant): "pk_cfg" (persistent GEMM tile: -1 auto, 0 128x128, 10 128x64,
 * 20 64x128, 30 64x64), "pk_elds" (-1 auto, 0/1 staged epilogue), "dw_lds" (1 = LDS-tiled depthwise conv),
 * "dw_rows" (its strip height), "attn_cfg" (stage-1 fused attention block tile: -1 auto, 4 = 8 waves x 512
 * queries, 6 = 4 waves x 256).  Initial values from SVK_PK_CFG / SVK_PK_ELDS / SVK_DW_LDS / SVK_DW_LR /
 * SVK_ATTN_CFG.  (Round 6: the timing-ablation switches that skipped work or stores — "pk_diag", "ffn_diag" —
 * exist only in a -DSVK_DIAG build of the library, never in the product .so.) */
int svk_tune(const char* knob, int value);

/* C[m, n] = act(sum_k A[m, k] * W[n, k] + bias[n]) + R[m, n]
 * Replaces nn.Linear (+ activation, + residual add) at: Attention q/kv/proj
 * (mix_transformer_evp.py:81-84, 112-128), Mlp fc1/fc2 (:37-40, 61-65), Block residuals
 * (:168-169), PromptGenerator embedding/lightweight/shared MLPs (:599-642, 752, 800-812),
 * SegFormerHead MLP/linear_fuse/fc (segformer_head.py:38-43, 74-80, 101-106),
 * MS-TCN 1x1 Conv1d (mstcn.py:161, 171), Transformer fc (adapter_transformer.py:327, 346).
 * bias, R may be NULL.  lda/ldw/ldr/ldc in elements. */
int svk_gemm(int dtype, const void* A, long lda, const void* W, long ldw, const float* bias,
             const void* R, long ldr, void* C, long ldc, int M, int N, int K, int act, void* stream);

/* Implicit-GEMM Conv2d over an NHWC input, weights packed [Cout][k][k][Cin]:
 * Y[b, oy, ox, co] = act(sum X[b, oy*s-p+i, ox*s-p+j, ci] * Wt[co, i, j, ci] + bias[co]) + R[...]
 * OH = (H + 2p - k)/s + 1.  Replaces OverlapPatchEmbed.proj (mix_transformer_evp.py:188-189,
 * 210), Attention.sr (:89, 116), PromptGenerator handcrafted convs (:582-595),
 * OpticalFlowEncoder conv+BN(eval, folded)+ReLU (:823-853). */
int svk_conv2d_nhwc(int dtype, const void* X, int B, int H, int W, int Cin, const void* Wt,
                    const float* bias, const void* R, void* Y, int Cout, int k, int stride, int pad,
                    int act, void* stream);

/* Sequence-reduction conv + LayerNorm, Y = LN(conv(X) + bias) (Attention.sr + Attention.norm,
 * mix_transformer_evp.py:115-117).  bf16 long-K patchify convs split K over svk_conv2d_ln_workspace()
 * bytes of caller-owned f32 workspace (0 = no split; ws may then be NULL) and reduce the parts inside
 * the LayerNorm; otherwise conv then in-place LayerNorm.  Y contiguous [B, OH, OW, Cout]. */
long svk_conv2d_ln_workspace(int dtype, int B, int H, int W, int Cin, int Cout, int k, int stride, int pad);
int svk_conv2d_ln_nhwc(int dtype, const void* X, int B, int H, int W, int Cin, const void* Wt, const float* bias,
                       const float* gamma, const float* beta, float eps, void* Y, int Cout, int k, int stride,
                       int pad, void* ws, long ws_bytes, void* stream);

/* Row LayerNorm: Y = (X - mean) / sqrt(var + eps) * gamma + beta over C channels.
 * Replaces every nn.LayerNorm on the path (mix_transformer_evp.py:90, 139-146, 190,
 * 245-269, 876). */
int svk_layernorm(int dtype, const void* X, long ldx, void* Y, long ldy, const float* gamma,
                  const float* beta, int M, int C, float eps, void* stream);

/* Multi-head softmax attention, per batch b and head h (columns h*hd .. h*hd+hd-1):
 * O = softmax(scale * Q K^T) V.  sb* = batch strides (elements).  Nk <= 256, hd <= 64.
 * Replaces Attention q@k^T/softmax/@v (mix_transformer_evp.py:123-127) and
 * nn.MultiheadAttention's core (:868-883). */
int svk_attention(int dtype, const void* Q, long ldq, long sbq, const void* K, long ldk, long sbk,
                  const void* V, long ldv, long sbv, void* O, long ldo, long sbo, int B, int Nq,
                  int Nk, int heads, int hd, float scale, void* stream);

/* Depthwise 3x3 conv (pad 1) + bias + activation over NHWC, taps w[9][C] (f32).
 * Replaces DWConv.forward + Mlp.act (mix_transformer_evp.py:24-30, 62-63). */
int svk_dwconv3x3(int dtype, const void* X, const float* w, const float* bias, void* Y, int B,
                  int H, int W, int C, int act, void* stream);

/* Whole MixFFN + Block residual (mix_transformer_evp.py:32-67, DWConv :19-30, Block :169) in one kernel,
 * optionally followed by the next LayerNorm (the stage norm :370-412):
 *   Y = X + fc2(GELU(dwconv3x3(fc1(XN)))),  Yn = LN(Y; gamma, beta, eps) when gamma != NULL (Y may
 *   then be NULL: only the normalised map is written)
 * over NHWC [B, H, W, C] bf16 / f16 maps; the 4C-wide hidden map never leaves the chip.  W1 [4C][C],
 * W2 [C][4C] in the map dtype; b1 [4C], b2 [C], gamma/beta [C] f32.  tpk = the depthwise taps and bias
 * packed per hidden channel quad q (channels 4q .. 4q+3) as 13 16-byte records: 12 for (dy, c) holding
 * the 32-bit pairs of the map dtype (w[dy][1], w[dy][2]), (w[dy][0], w[dy][1]), (0, w[dy][0]),
 * (w[dy][2], 0) of channel 4q + c (element 0 in the low half), then the 4 depthwise biases as f32
 * (svk.ops.mixffn_pack_taps).  All pointers 16-byte aligned.
 * Instantiated for the 224x224 MiT stage-1/2 shapes (svk_mixffn_supported(W, C)); SVK_EUNSUPPORTED
 * otherwise (callers then run svk_mixffn_fc1_dwconv + svk_gemm). */
int svk_mixffn_supported(int W, int C);
int svk_mixffn_fused(int dtype, const void* XN, const void* X, const void* W1, const float* b1, const void* tpk,
                     const void* W2, const float* b2, void* Y, void* Yn, const float* gamma, const float* beta,
                     float eps, int B, int H, int W, int C, void* stream);

/* The same whole MixFFN (+ LayerNorm) as svk_mixffn_fused, f16, with the depthwise window in registers
 * (csrc/mixffn_rw.hip: fc1's MFMA output layout is the conv layout — horizontal taps are neighbouring
 * lanes, vertical taps the rows a lane computed before — and the GELU output is fc2's MFMA operand;
 * the hidden channels split over the waves of a workgroup, whose fc2 partial sums meet in LDS once per
 * image row).  Same operands as svk_mixffn_fused except the depthwise conv: taps [9][4C] f32 (row
 * dy*3+dx) and dbias [4C] f32, rounded to f16 in the kernel.  Instantiated where
 * svk_mixffn_rw_supported(dtype, W, C) (the MiT-b1..b5 stage-1 shape: W = 56, C = 64, f16). */
int svk_mixffn_rw_supported(int dtype, int W, int C);
int svk_mixffn_rw(int dtype, const void* XN, const void* X, const void* W1, const float* b1, const float* taps,
                  const float* dbias, const void* W2, const float* b2, void* Y, void* Yn, const float* gamma,
                  const float* beta, float eps, int B, int H, int W, int C, void* stream);

/* Stage-1 patch embedding over space-to-depth blocks + its LayerNorm (csrc/stem.hip; OverlapPatchEmbed,
 * mix_transformer_evp.py:174-215): Y = LN(conv2x2(Xs, W) + bias) with Xs [B, HB, WB, CS] the s2d map
 * (svk_nchw_to_s2d / svk_gauss5x5_s2d), W [Cout][2][2][CS] (svk.pack.conv_w_s2d), gamma / beta [Cout] f32
 * (gamma = nullptr: no LayerNorm), Y [B, HB-1, WB-1, Cout].  Instantiated where
 * svk_conv2d_s2d_ln_supported(dtype, CS, Cout, OW) (16-bit, CS in {32, 48}, Cout = 64, OW <= 64). */
int svk_conv2d_s2d_ln_supported(int dtype, int CS, int Cout, int OW);
int svk_conv2d_s2d_ln(int dtype, const void* Xs, int B, int HB, int WB, int CS, const void* W, const float* bias,
                      const float* gamma, const float* beta, float eps, void* Y, int Cout, void* stream);

/* MixFFN back half for the stage-3 / stage-4 shapes (csrc/dwfc2.hip): Y = GELU(dwconv3x3(H) + dbias) W2^T + b2
 * (+ R), the depthwise output never written: each 64-token tile builds its GELU map per 64-channel K-step in
 * LDS from a halo'd H tile and runs the fc2 MFMAs on it (mix_transformer_evp.py:60-67, 24-30; replaces
 * svk_dwconv3x3 + svk_gemm).  H [B, Himg, Wimg, K] (fc1 output, 16-bit), taps [9][K] f32 (row dy*3+dx), dbias
 * [K] f32, W2 [N][K], b2 [N] f32, R / Y [B*Himg*Wimg][N]; H, W2, taps, dbias, b2 16-byte aligned, R / Y 8-byte.
 * Instantiated where svk_mixffn_dw_fc2_supported(dtype, W, N, K) (stages 3 / 4 of MiT-b1..b5 at 224x224:
 * 14 x 14 with N = 320, 7 x 7 with N = 512); SVK_EUNSUPPORTED otherwise. */
int svk_mixffn_dw_fc2_supported(int dtype, int W, int N, int K);
int svk_mixffn_dw_fc2(int dtype, const void* H, const float* taps, const float* dbias, const void* W2, const float* b2,
                      const void* R, void* Y, int B, int Himg, int Wimg, int K, int N, void* stream);

/* The stage-2 / 3 / 4 shapes (28 x 28 with N = 128, 14 x 14 with N = 320, 7 x 7 with N = 512; K % 64 == 0,
 * 16-bit) with the
 * depthwise conv on the matrix cores
 * (csrc/dwfc2.hip, dwrw): the operands are packed once per weight set — svk_mixffn_dw_fc2_pack writes
 * svk_mixffn_dw_fc2_packed_bytes(...) bytes (16-byte aligned): per 64-channel K-step the W2 fragments in load
 * order, then the taps rounded to the 16-bit type [9][K] and the dwconv biases [K] f32 (round 6: the kernel builds
 * its block-diagonal dwconv A fragments from those; the buffer size changed with that layout) —
 * then svk_mixffn_dw_fc2_packed computes Y = GELU(dwconv3x3(H) + dbias) W2^T + b2 (+ R) from H and the packed
 * buffer (same H / b2 / R / Y contract as svk_mixffn_dw_fc2).  packed_bytes is 0 where there is no packed form;
 * the other two return SVK_EUNSUPPORTED there. */
long svk_mixffn_dw_fc2_packed_bytes(int dtype, int W, int N, int K);
int svk_mixffn_dw_fc2_pack(int dtype, const float* taps, const float* dbias, const void* W2, int W, int N, int K,
                           void* packed, void* stream);
int svk_mixffn_dw_fc2_packed(int dtype, const void* H, const void* packed, const float* b2, const void* R, void* Y,
                             int B, int Himg, int Wimg, int K, int N, void* stream);
/* The same with the activation chosen: act = SVK_ACT_GELU (svk_mixffn_dw_fc2_packed) or SVK_ACT_NONE, i.e.
 * Y = (dwconv3x3(H) + dbias) W2^T + b2 (+ R) — with flipped taps, zero dbias and W2 = W1^T the data gradient of
 * a frozen MixFFN's DWConv + fc1 (train_evp.py's backward through mix_transformer_evp.py:60-62, svk/train.py).
 * 14 x 14 / N = 320 and 7 x 7 / N = 512 only for SVK_ACT_NONE. */
/* The training forward (round 6; act = SVK_ACT_GELU, 14 x 14 / 7 x 7): as svk_mixffn_dw_fc2_packed, plus U
 * (optional, [B][Himg][Wimg][K] 16-bit, 8-byte aligned) receives the pre-activation dwconv3x3(H) + dbias — the
 * GELU backward's source — and rscale (optional, f32) scales each token's fc2 output by rscale[token / rdiv]
 * before R is added (DropPath per frame: mix_transformer_evp.py:167-171 in train mode).  Replaces
 * svk_dwconv3x3 (pre-activation store) + svk_gemm (row scale, residual) in svk/train.py's block forward. */
int svk_mixffn_dw_fc2_packed_ex(int dtype, const void* H, const void* packed, const float* b2, const void* R,
                                void* Y, int B, int Himg, int Wimg, int K, int N, int act, void* U,
                                const float* rscale, int rdiv, void* stream);
int svk_mixffn_dw_fc2_packed_act(int dtype, const void* H, const void* packed, const float* b2, const void* R,
                                 void* Y, int B, int Himg, int Wimg, int K, int N, int act, void* stream);

/* GEMM + bias + residual + LayerNorm over the full output row in one kernel (csrc/gemm_ln.hip): X = A W^T + bias
 * (+ R) rounded to the 16-bit type, H = LayerNorm(X; gamma, beta, eps) — Block's x + proj(...) followed by norm2,
 * or the prompt adapter's x + shared_mlp(...) followed by norm1 (mix_transformer_evp.py:167-171, 776-815; replaces
 * svk_gemm + svk_layernorm).  16-bit, N in {320, 512}, K % 8 == 0.  W is consumed PACKED: svk_gemm_ln_pack writes
 * svk_gemm_ln_packed_bytes(dtype, N, K) bytes (0 where not instantiated) from W [N][K]; then svk_gemm_ln reads A
 * [M][K] (row-contiguous), the packed buffer, bias [N] / gamma [N] / beta [N] f32 (bias may be NULL), R / X / H
 * [M][N] (R and X may be NULL).  A, packed, bias, gamma, beta, X, H 16-byte aligned (X and H are stored as
 * 16-byte row chunks); R 8-byte. */
long svk_gemm_ln_packed_bytes(int dtype, int N, int K);
int svk_gemm_ln_pack(int dtype, const void* W, int N, int K, void* packed, void* stream);
int svk_gemm_ln(int dtype, const void* A, int M, int K, const void* packed, const float* bias, const void* R,
                const float* gamma, const float* beta, float eps, void* X, void* H, int N, void* stream);

/* MixFFN front half, G = act(dwconv3x3(XN W1^T + b1) + dbias) over NHWC maps (Mlp.fc1 -> DWConv -> GELU,
 * mix_transformer_evp.py:60-63, 24-30): the 4C-wide hidden map stays on chip (fc1 recomputed on one
 * halo row above / below each strip).  bf16, C in {32, 64, 128}, hidden % 64 == 0; W1 [hidden][C] bf16,
 * b1 [hidden], taps [9][hidden], dbias [hidden] f32; G [B, H, W, hidden]. */
int svk_mixffn_fc1_dwconv(int dtype, const void* XN, const void* W1, const float* b1, const float* taps,
                          const float* dbias, void* G, int B, int H, int W, int C, int hidden, int act, void* stream);
/* The same with C in {32, 64, 128, 320, 512} and an optional pre-activation output Gpre (dwconv3x3(...) +
 * dbias rounded to the storage type, before act; nullptr = none): the training forward's MixFFN front half,
 * whose GELU backward reads it (train_evp.py's frozen backbone: fc1's output itself is never needed). */
int svk_mixffn_fc1_dwconv_ex(int dtype, const void* XN, const void* W1, const float* b1, const float* taps,
                             const float* dbias, void* G, void* Gpre, int B, int H, int W, int C, int hidden,
                             int act, void* stream);

/* NCHW f32 -> NHWC dtype with the channel dim zero-padded to Cpad >= C (input packing of frames /
 * flow, view(-1,3,224,224) at :354; padding to 8 lets the first convs take the vector path). */
int svk_nchw_to_nhwc(int dtype_out, const float* X, void* Y, int B, int C, int H, int W, int Cpad,
                     void* stream);

/* GaussianFilter.conv_gauss (mix_transformer_evp.py:511-514): reflect-pad 2 + binomial 5x5/256,
 * NCHW f32 in -> NHWC dtype out, channels zero-padded to Cpad >= C. */
/* Stem input packing for the k = 7, stride-4 convs (OverlapPatchEmbed 1 and the flow encoder's conv1,
 * mix_transformer_evp.py:226-229, 838-840): NCHW f32 [B, C, H, W] -> space-to-depth blocks [B, NBH, NBW,
 * s*s*C] in dtype_out (block (by, bx) = input rows / columns s*by - pad .. s*by - pad + s - 1, channel
 * (dy*s + dx)*C + c, zeros outside the image), so the conv becomes a 2x2 stride-1 unpadded conv over the
 * blocks with NBH = OH + 1, NBW = OW + 1.  s = 4, C in {2, 3}, bf16 / f16. */
int svk_nchw_to_s2d(int dtype_out, const float* X, void* Y, int B, int C, int H, int W, int s, int pad, int NBH,
                    int NBW, void* stream);

/* GaussianFilter.conv_gauss (reflect pad 2, binomial 5x5 / 256; mix_transformer_evp.py:495-514) written as
 * the stem's space-to-depth blocks [B, NBH, NBW, 48] (svk_nchw_to_s2d's layout with 3 channels, channels
 * >= C zero): the handcrafted prompt stem's input.  Values bitwise equal to svk_gauss5x5_reflect's. */
int svk_gauss5x5_s2d(int dtype_out, const float* X, void* Y, int B, int C, int H, int W, int pad, int NBH, int NBW,
                     void* stream);

int svk_gauss5x5_reflect(int dtype_out, const float* X, void* Y, int B, int C, int H, int W, int Cpad,
                         void* stream);

/* Bilinear resize (align_corners=False) of NHWC token maps [B, H*W, C] (row stride ldx)
 * to [B, OH*OW, C] (row stride ldy).  Replaces resize() in SegFormerHead
 * (segformer_head.py:150-156). */
int svk_resize_bilinear(int dtype, const void* X, long ldx, void* Y, long ldy, int B, int H, int W,
                        int C, int OH, int OW, void* stream);

/* The head's pyramid resizes in one launch: nl (1-4) 16-bit levels X[l] ([B, H[l]*W[l], C[l]], row stride
 * ldx[l], C[l] % 8 == 0) each resized as svk_resize_bilinear to OH x OW and written side by side (level l at
 * channel offset C[0] + ... + C[l-1]) into Y [B, OH*OW, ldy].  Bit-identical to nl svk_resize_bilinear calls;
 * replaces SegFormerHead's four resize() calls before the channel concat (segformer_head.py:150-158). */
int svk_resize_bilinear_multi(int dtype, int nl, const void* const* X, const long* ldx, const int* H,
                              const int* W, const int* C, void* Y, long ldy, int B, int OH, int OW, void* stream);

/* Y[b, c] = mean_r X[b*R + r, c] (f32 out).  Replaces AdaptiveAvgPool2d + flatten
 * (segformer_head.py:167-169). */
int svk_mean_rows(int dtype, const void* X, long ldx, float* Y, int B, int R, int C, void* stream);

/* Row softmax over C channels (f32): MS-TCN inter-stage softmax over classes (mstcn.py:126). */
int svk_softmax_rows(const float* X, long ldx, float* Y, long ldy, int M, int C, void* stream);

/* One MS-TCN DilatedResidualLayer (mstcn.py:208-214) over a time-major [T, F] f32 map:
 * h = relu(sum_j Wd[j] x[t + off_j] + bd); y[t] = x[t] + W1 h + b1;
 * causal: off = (-2d, -d, 0); else (-d, 0, +d); out-of-range taps read zero.
 * Weights as transposed packs: WdT [3][F_in][F_out] (WdT[j][i][o] = conv_dilated.weight[o][i][j]),
 * W1T [F_in][F_out] (= conv_1x1.weight[:, :, 0]^T). F <= 64. */
int svk_mstcn_layer(const float* X, const float* WdT, const float* bd, const float* W1T,
                    const float* b1, float* Y, int T, int F, int dilation, int causal, void* stream);

/* Prompt adapter + norm1 of a MiT Block in one kernel (mix_transformer_evp.py:776-815 get_prompt, then
 * Block.norm1), C in {64, 128, 320} (stages 1-3), prompt width C4 = C / 4, bf16 / f16:
 * Xo = X + GELU(S Wl^T + bl) Ws^T + bs, Ho = LayerNorm(Xo; gamma1, beta1, eps).  S [M, C4], X / Xo / Ho [M, C]
 * contiguous; Wl [C4, C4], Ws [C, C4] (nn.Linear); bl / bs may be NULL. */
int svk_prompt_ln(int dtype, const void* S, const void* X, const void* Wl, const float* bl, const void* Ws,
                  const float* bs, const float* gamma1, const float* beta1, float eps, void* Xo, void* Ho, int M,
                  int C, void* stream);

/* Attention half of a MiT Block in one kernel for the 64-channel-head stages (mix_transformer_evp.py:71-131,
 * 134-171; C = 64 with one head (stage 1) or C = 128 with two heads (stage 2), sequence-reduced keys
 * Nk <= 64), bf16 / f16: q = Hn Wq^T + bq, o_h = softmax(scale q_h k_h^T) v_h, Y = X + o Wp^T + bp,
 * H2 = LayerNorm(Y; gamma2, beta2, eps).  Hn = norm1(X), X, Y, H2 contiguous [B, N, C]; KV [B, Nk, ldkv]
 * holds k | v (the kv Linear's output); Wq, Wp nn.Linear [C, C]; bq may be NULL. */
int svk_attn_block(int dtype, const void* Hn, const void* X, const void* KV, long ldkv, const void* Wq,
                      const float* bq, const void* Wp, const float* bp, const float* gamma2, const float* beta2,
                      float eps, void* Y, void* H2, int B, int N, int Nk, int C, float scale, void* stream);

/* Ragged batch of videos in one launch (trans_SV_output.py:251-291 and tecno.py's test loop run the
 * model video by video): X / Y hold the videos' [T_v, F] maps concatenated time-major; tiles is a
 * device table of ntiles int4 records {first row of the video, T_v, tile start t0 inside the video, 0},
 * one per svk_mstcn_tile_size() time steps of every video (16-byte aligned).  Per video the result
 * equals svk_mstcn_layer on that video alone (taps never cross a video boundary). */
int svk_mstcn_tile_size(void);
int svk_mstcn_layer_ragged(const float* X, const float* WdT, const float* bd, const float* W1T, const float* b1,
                           float* Y, const int* tiles, int ntiles, int F, int dilation, int causal, void* stream);

/* Training (tecno.py:195-259 trains MultiStageModel_S with nn.Dropout(p = 0.5) active in every
 * DilatedResidualLayer): Y = X + mask * (W1 relu(dilated conv) + b1) with mask values 0 or 1/keep;
 * H [T, F] receives relu(pre) for the backward. */
int svk_mstcn_layer_train(const float* X, const float* WdT, const float* bd, const float* W1T, const float* b1,
                          const float* mask, float* Y, float* H, int T, int F, int dilation, int causal, void* stream);
/* Backward of svk_mstcn_layer_train: dX = dY + conv^T(dPre), dPre = relu'(H) * (mask * dY) W1 (written to
 * the caller's dPre [T, F] scratch); dWd [F_out][F_in][3] (the nn.Conv1d weight layout), dbd, dW1 [F][F],
 * db1 += (f32 atomics: zero them).  Here Wd is packed [3][F_out][F_in] and W1 is conv_1x1.weight
 * [F_out][F_in]; ws: svk_mstcn_bwd_workspace(T, F) bytes (per-16-step-tile partial weight gradients). */
long svk_mstcn_bwd_workspace(int T, int F);
int svk_mstcn_layer_bwd(const float* X, const float* H, const float* mask, const float* dY, const float* Wd,
                        const float* W1, float* dPre, float* dX, float* dWd, float* dbd, float* dW1, float* db1,
                        float* ws, int T, int F, int dilation, int causal, void* stream);
/* Backward of the inter-stage softmax (mstcn.py:126): dX = P * (dP - rowsum(P * dP)) (+ R, may be NULL:
 * the stage's own output gradient). */
int svk_softmax_rows_bwd(const float* P, long ldp, const float* dP, long lddp, const float* R, long ldr, float* dX,
                         long lddx, int M, int C, void* stream);

/* CausalMambaModel (mstcn.py:282-343) block internals; the reference's Mamba is mamba_ssm's
 * `Mamba` (mamba_simple.py, imported at mstcn.py:9), absent from the reference snapshot.
 * Causal depthwise Conv1d (pad K-1, keep the first T outputs) + SiLU over B videos of T
 * time-major rows: Y[b*T+t, d] = silu(bias[d] + sum_k W[d, k] X[b*T + t-(K-1)+k, d]).
 * Replaces Mamba.conv1d + act (x = act(conv1d(x)[..., :seqlen])).  K <= 8, bias may be NULL. */
int svk_mamba_conv_silu(const float* X, long ldx, const float* W, const float* bias, float* Y, int B, int T,
                        int Di, int K, void* stream);

/* Selective scan (mamba_ssm selective_scan_fn with delta_bias, delta_softplus=True, z gate):
 * delta = softplus(Wdt[d,:] . XD[r, 0:R] + bdt[d]); h = exp(delta A[d,n]) h + delta XD[r, R+n] U[r,d];
 * Y[r,d] = (sum_n XD[r, R+N+n] h[n] + Dp[d] U[r,d]) * silu(Z[r,d]), rows r = b*T+t, state reset per
 * video.  U/Y [B*T, Di]; XD [B*T, >= R+2N] (x_proj output: dt_low | B | C); A = -exp(A_log) [Di, N];
 * Wdt [Di, R].  N in {16, 32, 64}, R <= 16. */
int svk_mamba_scan(const float* U, const float* XD, long ldxd, const float* Z, long ldz, const float* Wdt,
                   const float* bdt, const float* A, const float* Dp, float* Y, int B, int T, int Di, int N,
                   int R, int seg_len, float* ws, void* stream);
/* seg_len >= T: one sequential pass (ws may be NULL).  Otherwise time is split into ceil(T/seg_len)
 * segments (seg_len a multiple of 32) scanned concurrently in two passes; ws (caller-owned) holds
 * svk_mamba_scan_workspace(B, T, Di, N, seg_len) bytes of per-segment end states and delta sums. */
long svk_mamba_scan_workspace(int B, int T, int Di, int N, int seg_len);

/* Ragged batches of videos (tecno.py / trans_SV_output.py walk the test videos one by one): the videos'
 * rows are concatenated time-major.  conv: tpos[r] = time index of row r inside its video (the causal
 * taps stop at the video's first row).  scan: segs = nseg int4 records {first row of the video, T_v,
 * segment index z, index of the video's first record} (a video's records consecutive, 16-byte aligned),
 * segments of seg_len steps (a multiple of 32) scanned in two passes; ws = svk_mamba_scan_ragged_workspace
 * bytes.  Per video the result equals svk_mamba_conv_silu / svk_mamba_scan on that video alone. */
int svk_mamba_conv_silu_ragged(const float* X, long ldx, const float* W, const float* bias, float* Y,
                               const int* tpos, long rows, int Di, int K, void* stream);
int svk_mamba_scan_ragged(const float* U, const float* XD, long ldxd, const float* Z, long ldz, const float* Wdt,
                          const float* bdt, const float* A, const float* Dp, float* Y, const int* segs, int nseg,
                          int Di, int N, int R, int seg_len, float* ws, void* stream);
long svk_mamba_scan_ragged_workspace(int nseg, int Di, int N);
/* svk_mamba_scan that also stores the pre-gate output Yss = sum_n C h + D u [B*T, Di] (training). */
int svk_mamba_scan_train(const float* U, const float* XD, long ldxd, const float* Z, long ldz, const float* Wdt,
                         const float* bdt, const float* A, const float* Dp, float* Y, float* Yss, int B, int T,
                         int Di, int N, int R, int seg_len, float* ws, void* stream);
/* Selective-scan backward (tecno.py:256 loss.backward() through CausalMambaModel): from dOut [B*T, Di]
 * -> dU, dZ (row stride lddz), dS = d(softplus input) [B*T, Di] (the dt projection's gradients are GEMMs
 * on it), dXD columns R .. R+2N (dB | dC, += f32 atomics: zero them), dA (w.r.t. A = -exp(A_log)) [Di, N]
 * and dD [Di] (+=).  ws: svk_mamba_scan_bwd_workspace() bytes (state checkpoints). */
long svk_mamba_scan_bwd_workspace(int B, int T, int Di, int N);
int svk_mamba_scan_bwd(const float* U, const float* XD, long ldxd, const float* Z, long ldz, const float* Wdt,
                       const float* bdt, const float* A, const float* Dp, const float* Yss, const float* dOut,
                       float* dU, float* dZ, long lddz, float* dS, float* dXD, long lddxd, float* dA, float* dD,
                       int B, int T, int Di, int N, int R, float* ws, void* stream);
/* Backward of svk_mamba_conv_silu: dPre [B*T, Di] scratch, dX (row stride lddx) written, dW [Di, K] and
 * db [Di] += (db may be NULL). */
int svk_mamba_conv_silu_bwd(const float* X, long ldx, const float* W, const float* bias, const float* dY,
                            float* dPre, float* dX, long lddx, float* dW, float* db, int B, int T, int Di, int K,
                            void* stream);

/* Temporal-model training step (tecno.py:195-259).  Loss of tecno.py:237-254 over S stages of
 * time-major logits (stage s row t at logits + s * sstride + t * ld; columns 0..P-1 phase logits,
 * P..2P-1 anticipation regressions): loss[0] = (1/S) sum_s CrossEntropy(weight=class_w, 'mean'),
 * loss[1] = (1/S) sum_s SmoothL1('mean'), loss[2] = correct argmax count of the last stage; dlogits
 * (same layout) = d(loss[0] + loss[1]).  class_w may be NULL (unweighted). */
int svk_tecno_loss(const float* logits, long ld, long sstride, int S, int T, int P, const long* labels,
                   const float* ant_targets, const float* class_w, float* loss, float* dlogits, void* stream);
/* clip_grad_norm_ + torch.optim.AdamW over one flat f32 buffer.  svk_grad_sqnorm writes
 * svk_norm_parts() partial sums of squares and advances the device step counter (may be NULL when
 * the caller counts); svk_adamw scales g by min(max_norm / (||g|| + 1e-6), 1) (partials NULL or
 * max_norm <= 0: no clipping; the scaled g is written back), then applies AdamW with the learning
 * rate read from device memory (*lr) and bias corrections for step *step. */
int svk_norm_parts(void);
int svk_grad_sqnorm(const float* g, long n, float* partials, long long* step, void* stream);
int svk_adamw(float* p, float* g, float* m, float* v, long n, const float* partials, float max_norm,
              const float* lr, float beta1, float beta2, float eps, float weight_decay, const long long* step,
              void* stream);
/* Y = -exp(X) (f32): the selective scan's A = -exp(A_log) after each optimizer step. */
int svk_neg_exp(const float* X, float* Y, long n, void* stream);

/* Relaxed-boundary phase metrics (eval_and_vis.py:35-161) over V videos of int64
 * labels concatenated in gt / pred with offsets [V + 1]: counts [V][2 + 4P] = (T, #forgiven-diff-zero,
 * then per phase (TP over the gt|pred union, |union|, #pred, #gt)); exact integers, the caller forms the
 * reference's ratios.  P <= 16, one workgroup per video. */
int svk_phase_metrics(const long long* gt, const long long* pred, const long long* offsets, int V, int P,
                      int tolerance, long long* counts, void* stream);

/* Frame preprocessing: generate_evp_LFB.py:243-247's Resize((OH, OW)) ->
 * CenterCrop -> ToTensor -> Normalize on decoded uint8 RGB frames [B, H, W, 3], bit-exact to Pillow's
 * 8-bit bilinear resampling (libImaging/Resample.c: horizontal then vertical pass, 22-bit fixed-point
 * coefficients, round + clip to uint8 after each pass) and torch's f32 (u8 / 255 - mean) / std.
 * xbounds [OW, 2] / ybounds [OH, 2] = (first tap, tap count), xcoef [OW, ksx] / ycoef [OH, ksy]: Pillow's
 * fixed-point coefficients (device arrays, built by svk/preproc.py); only the CH x CW crop window at
 * (crop_y0, crop_x0) of the resized frame is produced.  tmp: caller-owned [B, H, CW, 3] uint8 scratch.
 * out [B, 3, CH, CW] f32.  mean / std: HOST arrays of 3 floats. */
int svk_frame_preproc(const void* frames, void* tmp, float* out, const int* xbounds, const int* xcoef, int ksx,
                      const int* ybounds, const int* ycoef, int ksy, int B, int H, int W, int crop_y0,
                      int crop_x0, int CH, int CW, const float* mean, const float* std, void* stream);

/* Optical-flow transform (data_process.py:425-447 + CenterCrop): cv2.resize(INTER_LINEAR) of float32
 * flow [B, H, W, 2] to the (OH, OW) grid, u *= scale_u (= OW / W), v *= scale_v (= OH / H), crop CH x CW at
 * (crop_y0, crop_x0) -> out [B, 2, CH, CW] f32.  xofs/xalpha [OW] / [OW, 2] and yofs/yalpha: cv2's source
 * index and (1 - f, f) weights per output coordinate (device arrays, svk/preproc.py).  No FMA contraction. */
int svk_flow_preproc(const float* flow, float* out, const int* xofs, const float* xalpha, const int* yofs,
                     const float* yalpha, int B, int H, int W, int crop_y0, int crop_x0, int CH, int CW,
                     float scale_u, float scale_v, void* stream);

/* Training augmentations (train_evp.py:146-163 via data_process.py:53-186; replaces the DataLoader workers'
 * PIL transform of CholecFlowDataset.__getitem__, data_process.py:455-462): decoded uint8 frames / RGB segmaps
 * [B, H, W, 3] -> Pillow bilinear Resize to RH x RW -> RandomCrop CH x CW at (params[b*16+0], params[b*16+1]) ->
 * [ColorJitter] -> [flip] -> [rotate] -> ToTensor -> Normalize -> out [B, 3, CH, CW] f32, bit-exact to Pillow.
 * params [B][16] int32: x1, y1, flip, rot, a0..a5 (Image.rotate's inverse matrix in 16.16 fixed point), jitter,
 * brightness, contrast, saturation (f32 bits), hue shift (0..255), unused.  Workspace: tmp [B, H, CW, 3] uint8,
 * crop [B, CH, CW, 3] uint8, sums [B] int64.  Resize tables as svk_frame_preproc (for H -> RH, W -> RW). */
int svk_train_augment(const void* frames, void* tmp, void* crop, long long* sums, float* out, const int* xbounds,
                      const int* xcoef, int ksx, const int* ybounds, const int* ycoef, int ksy, const int* params,
                      int B, int H, int W, int RH, int RW, int CH, int CW, const float* mean, const float* std,
                      void* stream);

/* The geometric training augmentations on the RAFT flow (data_process.py:471-487): cv2 INTER_LINEAR resize +
 * displacement scale (tables as svk_flow_preproc), RandomCrop at (x1, y1), [flip: u negated], [rotate: nearest
 * affine grid sample + vector rotation] -> out [B, 2, CH, CW] f32.  params [B][16] int32: x1, y1, flip, rot, t00,
 * t01, t02, t10, t11, t12 (the grid's rescaled inverse rotation, f32 bits), cos, sin (f32 bits). */
int svk_train_augment_flow(const float* flow, float* out, const int* xofs, const float* xalpha, const int* yofs,
                           const float* yalpha, const int* params, int B, int H, int W, int CH, int CW, float scale_u,
                           float scale_v, void* stream);

/* Phase-anticipation targets (generate_phase_anticipation.py:10-34, generate_anticipation_gt): phases
 * [P, T] int64 one-hot presence (row stride ldp), horizon in minutes -> out [T, P] f32; per phase a
 * backward recurrence count = present ? 0 : min(horizon, count + 1/1500) in double, out = f32(count) / f32(horizon). */
int svk_anticipation_gt(const long long* phases, long ldp, int P, int T, double horizon, float* out, void* stream);

/* Causal window unfold (adapter_transformer.py:336-343 as pad + unfold):
 * Y[t, i, c] = X[t - len + 1 + i, c] (0 if negative) + pos[i, c] (pos may be NULL). */
int svk_window_unfold(int dtype, const void* X, long ldx, const float* pos, void* Y, int T, int C,
                      int len, void* stream);

/* Y[r, c] = X[r, c] + P[r % period, c] over M contiguous rows of C (P f32): the fixed
 * position table added to Transformer2_3_1's encoder input (build-defined, parity unpinned). */
int svk_add_bcast(int dtype, const void* X, const float* P, void* Y, long M, int C, int period, void* stream);

/* Elementwise dtype conversion (n elements). */
int svk_cast(int dtype_in, const void* X, int dtype_out, void* Y, long n, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Training step (train_evp.py:473-515): the frozen-backbone step differentiates through every
 * backbone block (prompts are injected at each block) and produces f32 gradients for the
 * trainable modules (head, prompt_generator, flow_encoder, cross_attn_s3/s4, :379-382).
 * Activation gradients are in the compute dtype; parameter gradients, statistics and optimizer
 * state are f32.  Gradient outputs marked "+=" accumulate (f32 atomics): the caller zeroes them.
 * ------------------------------------------------------------------------------------------- */

/* svk_dwconv3x3 that also stores the pre-activation map (Ypre, may be NULL) for the GELU backward. */
int svk_dwconv3x3_ex(int dtype, const void* X, const float* w, const float* bias, void* Y, void* Ypre, int B,
                     int H, int W, int C, int act, void* stream);

/* svk_gemm plus (a) a per-row scale s[m / rows_per_scale] applied to act(A W^T + bias) before the
 * residual add: timm DropPath (stochastic depth, mix_transformer_evp.py:168-169 in train mode) fused
 * into the branch GEMM and its adjoint in the data-gradient GEMM; (b) an activation backward
 * v *= uact'(U[m, n]) (U may be NULL): GELU/ReLU derivatives fused into the data-gradient GEMM. */
int svk_gemm_ex(int dtype, const void* A, long lda, const void* W, long ldw, const float* bias,
                const float* row_scale, int rows_per_scale, const void* U, long ldu, int uact,
                const void* R, long ldr, void* C, long ldc, int M, int N, int K, int act, void* stream);

/* Adjoint of a k = s patchify conv (Attention.sr, mix_transformer_evp.py:89, 116): GEMM rows are the
 * [B, H/s, W/s] patches, columns (i, j, ci), stored straight into the NHWC map Y [B, H, W, C]
 * (+ R at the same positions; R may alias Y).  K = Cout, W packed [(i, j, ci)][co]. */
int svk_gemm_unpatchify(int dtype, const void* A, long lda, const void* W, long ldw, const void* R, void* Y,
                        int B, int H, int Wd, int s, int C, int K, void* stream);

/* Skinny bf16 / f16 GEMM for the prompt path (PromptGenerator Linears, mix_transformer_evp.py:749-815):
 * C = act(A W^T + bias) * uact'(U) + R with N <= 64, K <= 128 (W held in LDS, A streamed in the MFMA
 * operand layout); same semantics as svk_gemm_ex without row scale.  A 16-byte aligned. */
int svk_gemm_skinny(int dtype, const void* A, long lda, const void* W, long ldw, const float* bias, const void* U, long ldu,
                    int uact, const void* R, long ldr, void* C, long ldc, int M, int N, int K, int act,
                    void* stream);

/* Skinny bf16 weight gradient: dW[N, K] += dY^T X, db[N] += colsum(dY) for N, K <= 128 with
 * ceil(N/16) * ceil(K/16) <= 16 (rounded to powers of two). */
int svk_wgrad_skinny(const void* dY, long ldy, const void* X, long ldx, float* dW, long lddw, float* db, int M,
                     int N, int K, void* stream);

/* dW[n, k] += sum_m dY[m, n] * X[m, k] and db[n] += sum_m dY[m, n] (db may be NULL)
 * (f32, split-M MFMA with atomics): nn.Linear weight and bias gradients. */
int svk_gemm_wgrad(int dtype, const void* dY, long ldy, const void* X, long ldx, float* dW, long lddw,
                   float* db, int M, int N, int K, void* stream);

/* Conv2d weight gradient: dW[Cout][kh][kw][Cin] (packed like the forward weights) += im2col(X)^T dY,
 * db[Cout] += column sums of dY (db may be NULL). */
int svk_conv2d_wgrad_nhwc(int dtype, const void* X, int B, int H, int W, int Cin, const void* dY,
                          int Cout, int k, int stride, int pad, float* dW, float* db, void* stream);

/* Conv2d data gradient (transposed-conv gather, power-of-two stride): dX [B,H,W,Cin] = col2im(dY) .
 * Wd packed [Cin][kh][kw][Cout]; optional R is added (R may alias dX). */
int svk_conv2d_dgrad_nhwc(int dtype, const void* dY, int B, int OH, int OW, int Cout, const void* Wd,
                          const void* R, void* dX, int H, int W, int Cin, int k, int stride, int pad,
                          void* stream);

/* [B*PH*PW, s*s*C] patch rows -> NHWC [B, PH*s, PW*s, C] (adjoint of the k = s patchify conv's im2col;
 * accumulate != 0 adds into Y). */
int svk_unpatchify(int dtype, const void* P, void* Y, int B, int PH, int PW, int s, int C, int accumulate,
                   void* stream);

/* Conv data gradient, second half (train_evp.py's loss.backward through the frozen OverlapPatchEmbed convs,
 * mix_transformer_evp.py:226-241, and the trainable handcrafted-prompt convs): P [B*OH*OW, k*k*Cin] holds
 * the per-tap products dY Wc^T (Wc [(ky, kx, ci), co]); dX NHWC [B, H, W, Cin] = the sum of the taps that
 * reached each input pixel, + R if non-null.  bf16 / f16, Cin % 8 == 0. */
int svk_col2im_nhwc(int dtype, const void* P, const void* R, void* dX, int B, int H, int W, int Cin, int OH, int OW,
                    int k, int stride, int pad, void* stream);

/* Scaled-dot-product attention backward (recomputes P): dQ, dK, dV written in the compute dtype
 * (dK/dV [B, Nk, heads*hd] with row stride lddk and batch stride sbdk).  bf16 with hd % 8 == 0,
 * hd <= 64, Nk <= 256: MFMA path (dQ kernel that also stores P and scale*dS, then batched MFMA
 * reductions dK = dS^T Q, dV = P^T dO); otherwise an LDS scalar path.  ws: caller-owned scratch of
 * at least svk_attention_bwd_workspace(...) bytes.  Replaces autograd through
 * mix_transformer_evp.py:123-127 and nn.MultiheadAttention (:868-883) in train_evp.py:512. */
long svk_attention_bwd_workspace(int dtype, int B, int Nq, int Nk, int heads, int hd);
int svk_attention_bwd(int dtype, const void* Q, long ldq, long sbq, const void* K, long ldk, long sbk,
                      const void* V, long ldv, long sbv, const void* O, long ldo, long sbo,
                      const void* dO, long lddo, long sbdo, void* dQ, long lddq, long sbdq, void* dK,
                      void* dV, long lddk, long sbdk, void* ws, long ws_bytes, int B, int Nq, int Nk, int heads,
                      int hd, float scale, void* stream);

/* LayerNorm backward (recomputes mean/rstd from X): dX = LN'(dY) (+ dR); dgamma/dbeta += (both or
 * neither; NULL for frozen norms).  C <= 512. */
int svk_layernorm_bwd(int dtype, const void* X, long ldx, const void* dY, long ldy, const float* gamma,
                      const void* dR, long ldr, void* dX, long lddx, float* dgamma, float* dbeta, int M, int C,
                      float eps, void* stream);

/* dX = dY * act'(U) (+ dR), elementwise over n (GELU erf / ReLU / tanh). */
int svk_act_bwd(int dtype, const void* U, const void* dY, const void* dR, void* dX, long n, int act, void* stream);

/* Column sums (and sums of squares, optional) over M rows, += into f32 sum/sumsq: batch statistics.
 * Deterministic (round 5): per-block partials into the caller's workspace ws, then a fixed-order sum — no
 * atomics, so the batch statistics (and every BN + ReLU gate after them) are bit-reproducible run to run.
 * ws holds svk_stats_ws_floats(M, C) floats (shared by svk_colstats and svk_bn_bwd). */
long svk_stats_ws_floats(int M, int C);
int svk_colstats(int dtype, const void* X, long ldx, int M, int C, float* sum, float* sumsq, float* ws,
                 void* stream);
/* The same statistics written, not accumulated: sums[0..C) = column sums, sums[C..2C) = sums of squares
 * (no zero-fill of the outputs needed before the call). */
int svk_colstats_set(int dtype, const void* X, long ldx, int M, int C, float* sums, float* ws, void* stream);

/* BatchNorm2d train mode on [M = B*H*W, C]: Y = act((X - mean) rsqrt(var + eps) g + b) from colstats
 * sums (biased variance), and its backward with the optional ReLU recomputed from X (dgamma/dbeta +=;
 * the same deterministic two-phase reduction through ws). */
int svk_bn_apply(int dtype, const void* X, const float* sum, const float* sumsq, const float* gamma,
                 const float* beta, void* Y, int M, int C, float eps, int act, void* stream);
int svk_bn_bwd(int dtype, const void* X, const void* dY, const float* sum, const float* sumsq,
               const float* gamma, const float* beta, void* dX, float* dgamma, float* dbeta, int M, int C,
               float eps, int relu, float* ws, void* stream);
/* running_mean/var momentum update (unbiased variance), as nn.BatchNorm2d does in train mode. */
int svk_bn_update_running(const float* sum, const float* sumsq, int M, int C, float momentum,
                          float* running_mean, float* running_var, void* stream);

/* Adjoint of svk_resize_bilinear: dX (f32 [B, H*W, C], +=) from dY [B, OH*OW, C] (row stride ldy). */
int svk_resize_bilinear_bwd(int dtype, const void* dY, long ldy, float* dX, int B, int H, int W, int C,
                            int OH, int OW, void* stream);

/* Adjoint of svk_mean_rows (+ Dropout2d mask): dY[b*R + r, c] = dF[b, c] * mask[b, c] * scale. */
int svk_bcast_rows(int dtype, const float* dF, const float* mask, float scale, void* dY, int B, int R, int C,
                   void* stream);

/* Y[r, c] = X[r, c] * s[r / rows_per]; y = a * b (f32). */
int svk_row_scale(int dtype, const void* X, const float* s, void* Y, long M, int C, int rows_per, void* stream);
int svk_mul_f32(const float* a, const float* b, float* y, long n, void* stream);

/* Counter-based Bernoulli(keep) mask scaled by 1/keep (values 0 or 1/keep): DropPath / Dropout2d.
 * counter (device int64, may be NULL) is mixed into the seed at run time (graph replays). */
int svk_keep_mask(float* out, long n, float keep, unsigned seed, const long long* counter, void* stream);
/* nm keep masks of n floats each in one launch: out[m*n + e] is element e of svk_keep_mask(keeps[m], seeds[m])
 * (keeps / seeds: device arrays of nm entries) — the step's DropPath masks (train_evp.py's drop_path_rate
 * schedule over the blocks, mix_transformer_evp.py:150-171) without one launch per mask. */
int svk_keep_mask_multi(float* out, long n, int nm, const float* keeps, const unsigned* seeds,
                        const long long* counter, void* stream);

/* CrossEntropyLoss(sum) + SmoothL1Loss(sum) (train_evp.py:390-391, 500-509): loss[0] += CE,
 * loss[1] += SmoothL1; dlogits / dant are the gradients of their sum. */
int svk_phase_loss(const float* logits, const float* ant, const long* labels, const float* ant_targets, int B,
                   int K, float* loss, float* dlogits, float* dant, void* stream);

/* torch.optim.SGD step (momentum, dampening, weight decay, nesterov; train_evp.py:405-419) over a
 * flat f32 parameter buffer; first != 0 initialises the momentum buffer. */
int svk_sgd(float* p, const float* grad, float* buf, long n, float lr, float momentum, float dampening,
            float wd, int nesterov, int first, void* stream);

/* Batched strided gather f32 master parameters -> packed compute-dtype views (one launch refreshes
 * all forward/transposed packs after an optimizer step).  desc: device array of
 * {long src, dst; int n[4]; long s[4]; int lim[4]; long start} (see csrc/train.hip PackDesc). */
int svk_pack_params(int dtype, const void* desc, int ndesc, long total, const float* src, void* dst,
                    void* stream);
/* svk_pack_params with 8 packed elements per thread (one 16-byte store): every descriptor's start (in the
 * linear index space) and its packed offset are multiples of 8, total % 8 == 0, dst 16-byte aligned; the
 * elements between a tensor's end and its 8-aligned slot end are written as zeros. */
int svk_pack_params8(int dtype, const void* desc, int ndesc, long total, const float* src, void* dst,
                     void* stream);

/* The transposed 2-D packs of the same refresh (dst[k * N + n] = src[n * K + k] for a row-major [N, K] f32
 * master matrix): tiles of 64 x 64 through LDS so both the master reads and the packed writes are
 * coalesced.  tiles: device array of ntiles {long src, dst; int K, N, n0, k0} (one per tile). */
int svk_pack_transpose(int dtype, const void* tiles, int ntiles, const float* src, void* dst, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SVK_H */
