/*
 * rdeic_hip.h — C ABI of librdeic_hip.so, the MI355X (gfx950) native library
 * behind the RDEIC relay-diffusion codec hot path.
 *
 * Plain C: raw pointers, sizes and an opaque hipStream_t (passed as void*).
 * No torch types cross this boundary. Device buffers are owned by the caller;
 * kernel launchers never allocate, never synchronise, and are capturable into
 * a hipGraph. Every export returns 0 on success or a negative errno-style code:
 *   -22 (EINVAL)  bad shape/argument      -28 (ENOSPC)  output capacity too small
 *   -74 (EBADMSG) corrupt / truncated bitstream      -5  kernel launch failure
 *
 * What each group replaces in the reference (ShreyasBhaktharam/RDEIC):
 *   conv / linear  : every nn.Conv2d / nn.Linear on the path (ldm/modules/diffusionmodules/
 *                    openaimodel.py:162-274, model.py:92-151, attention.py:153-203,
 *                    model/layers/res_blk.py:6-93, model/compression_modules.py:7-104)
 *   group/layer norm: GroupNorm32 (ldm/modules/diffusionmodules/util.py:224-226),
 *                    Normalize (attention.py:96-97, model.py:48-49), nn.LayerNorm (attention.py:265-267)
 *   attention      : CrossAttention.forward (attention.py:171-203), AttnBlock.forward (model.py:181-205)
 *   entropy model  : utils/ckbd.py:47-115 + compressai GaussianConditional.build_indexes/quantize
 *   coders         : compressai.ans.BufferedRansEncoder / RansDecoder (called at model/compression.py:166,
 *                    205-206, 230-231; utils/ckbd.py:103,112), compressai._CXX.pmf_to_quantized_cdf
 *                    (via GaussianConditional.update, compression.py:275-280), torchac.encode_float_cdf /
 *                    decode_float_cdf (utils/ckbd.py:130-141)
 */
#ifndef RDEIC_HIP_H
#define RDEIC_HIP_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ info */
int rdeic_version(void);
/* number of exported entry points this build provides (sanity check for loaders) */
int rdeic_abi_count(void);

/* ------------------------------------------------------- conv / linear
 * Implicit-GEMM convolution over NHWC activations (Linear == 1x1 conv over tokens).
 * out[p, co] = act( sum_k A[p,k] W[co,k] + bias[co] + emb[img(p), co] ) + res[p, co]
 * A is gathered on the fly from up to two channel-concatenated inputs, optionally
 * through a fused nearest-x2 upsample and a fused GroupNorm-affine(+SiLU) prologue.
 * Weights are packed [cout][wld] with wld = round_up(kh*kw*cin, 64), zero tail.
 */
typedef struct rdeic_conv_desc {
  const void* in0;      /* NHWC, pixel stride ld0 (elements) */
  const void* in1;      /* second concat segment or NULL */
  int32_t c0, c1;       /* channels of each segment (c1 = 0 when in1 == NULL) */
  int32_t ld0, ld1;
  int32_t n, h, w;      /* input batch / spatial size (before the fused upsample) */
  int32_t up2;          /* 1: nearest x2 upsample of the input is fused into the gather */
  const void* weight;   /* [cout][wld], compute dtype */
  int32_t wld;
  const float* bias;    /* [cout] or NULL */
  int32_t cout, kh, kw, stride, pad_t, pad_l;
  int32_t ho, wo;       /* output spatial size (before pixel shuffle) */
  const float* gn_ab;   /* NULL or [n][c0+c1][2] per-image channel affine from rdeic_groupnorm_stats */
  int32_t gn_silu;      /* 1: SiLU after the affine */
  const float* emb;     /* NULL or [n][emb_ld] per-(image, cout) additive term */
  int32_t emb_ld;
  int32_t act;          /* 0 none, 1 leaky_relu(act_param), 2 gelu (erf), 3 silu */
  float act_param;
  const void* res;      /* NULL or residual, same indexing/dtype as out, pixel stride res_ld */
  int32_t res_ld;
  void* out;
  int32_t out_ld;       /* pixel stride of out (elements) */
  int32_t out_mode;     /* 0 NHWC, 1 fused PixelShuffle(2): out is [n][2ho][2wo][cout/4],
                           2 fused GEGLU (attention.py:49-56): weight rows interleaved as 4 value / 4 gate,
                           out[p][cout/2] = x * gelu_erf(gate); bf16, LDS-DMA-eligible shapes, no res/emb/act */
  int32_t dtype;        /* 0 fp32 (parity mode), 1 bf16 (fp32 accumulate) */
  int32_t out_f32;      /* bf16 mode only: write fp32 output (and read fp32 residual) */
  int32_t batch;        /* >1: batched GEMM (grid z); operand z starts at +z*{in,w,out}_bs elements */
  int64_t in_bs, w_bs, out_bs;
  float* gn_part;       /* NULL, or GroupNorm statistics of the output in the partial format of
                           rdeic_groupnorm_parts_ab (rdeic_groupnorm_parts_floats(n*ho*wo, cout, gn_hw)
                           floats): fused into the LDS-DMA epilogue where the tile allows, else written
                           by a separate pass. out_mode 0, batch 1 */
  int32_t gn_hw;        /* pixels per image of the GroupNorm those statistics feed (divides n*ho*wo;
                           differs from ho*wo when a linear's rows are an image's tokens) */
  int32_t reserved;
  /* LayerNorm folded into a linear (bf16, out_mode 0 / 2, batch 1; attention.py:273-285 norm1/2/3 ->
   * to_q/k/v / to_q / ff.net.0.proj): the GEMM runs on the RAW rows x with weights diag(gamma) W and
   * the epilogue computes, before the bias, v = rstd_m * (acc - mean_m * ln_colsum[n]);
   * bias = bias + W beta. ln_rows: [M][2] fp32 (mean, rstd) from rdeic_layernorm_rowstats,
   * ln_colsum: [cout] fp32 column sums of the packed bf16 weight. NULL: off. */
  const float* ln_rows;
  const float* ln_colsum;
} rdeic_conv_desc;

int rdeic_conv2d(const rdeic_conv_desc* d, void* stream);
/* rdeic_conv2d with an explicit tile. Register-staged tiles (any bf16 conv without a GN
 * prologue): 0 256x256/16 waves, 1 256x128/8, 2 128x256/8, 3 128x128/4, 4 64x128/4,
 * 6 256x128/16, 7 128x256/16, 8 128x128/8, 9 128x128/16, 10 64x128/8. LDS-DMA tiles (bf16, both
 * concat segments multiples of 64 channels; other shapes fall back to the register path):
 * 21 256x128/8, 22 128x256/8, 23-24 128x128/4, 25 128x128/8, 26 64x128/4,
 * 27 128x128/8, 28 256x128/8, 29 128x256/8, 30 64x128/4, 31 128x64/4, 32 256x256/16,
 * 33 256x128/16, 34 128x128/16, 35 512x128/16, 36 64x128/8, 37 128x160/4, 38 64x160/4
 * (ring depths in conv_dma.hip). -1 = heuristic.
 * All tiles give
 * bit-identical results (same k order, same MFMA), so a caller may autotune. */
int rdeic_conv2d_tile(const rdeic_conv_desc* d, int32_t tile, void* stream);
/* Split-K variant for small-M / large-K layers (the UNet's 8x8 and 16x16 levels): `splits`
 * k-ranges accumulate into the caller's workspace, then a reduction sums them in split order
 * (deterministic) and applies bias / emb / act / residual. ws: >= splits * n*ho*wo * cout fp32 partials.
 * bf16 or fp32, no GN prologue, out_mode 0, batch 1, cout % 8 == 0. Not bit-identical to
 * rdeic_conv2d (different k grouping): not for the entropy-model nets. */
int rdeic_conv2d_splitk(const rdeic_conv_desc* d, int32_t splits, float* ws, size_t ws_floats, void* stream);
/* 2 (default): bf16 convs without a GN prologue pick among the big register-staged tiles
 * (256x256 / 256x128 / 128x256 / 128x128 / 64x128 / 128x64); 0: the 128-tile kernel with the
 * fused GroupNorm prologue everywhere (A/B timing, debugging). Results are bit-identical.
 * Returns the previous value. */
int rdeic_set_conv_path(int32_t path);
/* Tuning switches (process-wide). key 0: LDS-staged vector epilogue on (1, default) / off (0);
 * key 1: transposed head-dim-64 attention kernel on (1, default) / off (0);
 * key 3: XOR-swizzled 128-byte LDS rows on the <= 8-wave conv tiles (1 default) / padded rows (0);
 * key 4: force the big-tile candidate (0 256x256, 1 256x128, 2 128x256, 3 128x128, 4 64x128,
 *        5 128x64; -1 = automatic choice, default) — tuning only;
 * key 5: LDS-DMA conv kernel for 64-channel-aligned layers on (1, default) / off (0);
 * key 6: halo-strip 3x3 conv with the GroupNorm applied in LDS: 0 off, 1 GroupNorm-input convs
 *        (default), 2 every eligible conv (its k order differs from the im2col tiles');
 * key 8: head-dim-512 attention: 2 wave pairs splitting d over 32 queries (default, for L >= 4096:
 *        a per-image rule, so outputs stay batch-invariant), 1 one wave per 16 queries everywhere
 *        (fp32-rounding-level differences);
 * key 9: the halo conv's 8-row form (one 1024-thread block per CU, 8-slot weight ring) where the
 *        output height is a multiple of 8 and the epilogue is bf16 without emb / activation: 1 on
 *        (default), 0 the 4-row form everywhere (bit-identical outputs);
 * key 10: the VAE edge convs (conv_edge.hip): conv_in from 8 input channels on direct-load MFMA fragments
 *        (bit-identical to the register tile) and norm -> SiLU -> conv to <= 16 channels (fp32 rounding of the
 *        sums differs from the tiny-cout kernel): 1 on (default), 0 off.
 * Returns the previous value, or -22 for an unknown key. Results are bit-identical either way
 * (keys 0-5; 6 and 8 change fp32 rounding only). */
int rdeic_set_conv_option(int32_t key, int32_t value);

/* --------------------------------------------------------- normalisation
 * GroupNorm statistics over NHWC x[n][hw][ld] (first c channels), groups of c/g
 * contiguous channels; writes the per-(image, channel) affine
 *   ab[n][c][0] = gamma[c] * rstd(n,g),  ab[n][c][1] = beta[c] - mean(n,g) * ab[n][c][0]
 * so that consumers apply y = x*a + b (optionally SiLU) inside their own loads.
 * ws: fp32 workspace of at least rdeic_groupnorm_ws_floats(n, hw, c) floats. */
size_t rdeic_groupnorm_ws_floats(int32_t n, int32_t hw, int32_t c);
/* The input is the channel concatenation of x0 [n][hw][ld0] (c0 ch) and, if c1 > 0, x1 (c1 ch). */
/* GroupNorm affine from per-row-block partial sums (rdeic_conv_desc.gn_part): a 16-byte header
 * whose first int32 is R = 64 (rows per partial; hw % 64 == 0), then [rows/64][c][2] fp32 (sum,
 * sum of squares) in a canonical order independent of the conv tile (so the result is identical for
 * every tile and batch size). Channels [0, c0) from p0, [c0, c0+c1) from p1 (a concat); sums in
 * fp64 in a fixed order, var = E[x^2] - mean^2; writes ab like rdeic_groupnorm_stats.
 * rdeic_groupnorm_parts_floats: buffer size for a [rows][c] tensor, 0 when hw % 64 != 0. */
size_t rdeic_groupnorm_parts_floats(int64_t rows, int32_t c, int32_t hw);
int rdeic_groupnorm_parts_ab(const float* p0, int32_t c0, const float* p1, int32_t c1, int32_t n, int32_t hw,
                             int32_t groups, float eps, const float* gamma, const float* beta, float* ab,
                             void* stream);
int rdeic_groupnorm_stats(const void* x0, int32_t c0, int32_t ld0, const void* x1, int32_t c1, int32_t ld1,
                          int32_t n, int32_t hw, int32_t groups, float eps, const float* gamma, const float* beta,
                          float* ab, float* ws, int32_t dtype, void* stream);
/* y = silu?(x*a + b) * out_mul materialised (NHWC), where the consumer is not a conv
 * (e.g. the VAE encoder's c = swish(norm_out(h)), followed by the 0.18215 latent scale). */
/* GroupNorm finalize + apply in one launch for small images (hw = 64, 128 or 256 pixels: the UNet's 16^2 / 8^2
 * levels; openaimodel.py:200-204, 254-274; attention.py:250-266): y[n][hw][c0 + c1] = silu?(x * a + b) of the
 * channel concat of x0 (c0 ch, partials p0) and x1 (c1 ch, partials p1), the (a, b) table recomputed per block from
 * the partials (rdeic_groupnorm_parts_ab's arithmetic: bit-identical to parts_ab + apply) and also written to ab
 * [n][c][2]. bf16, c0 / c1 / ld / yld multiples of 8, c <= 2560, groups <= 256. */
int rdeic_groupnorm_parts_apply(const float* p0, int32_t c0, const float* p1, int32_t c1, const void* x0, int32_t ld0,
                                const void* x1, int32_t ld1, int32_t n, int32_t hw, int32_t groups, float eps,
                                const float* gamma, const float* beta, int32_t silu, float* ab, void* y, int32_t yld,
                                void* stream);
int rdeic_groupnorm_apply(const void* x, int32_t n, int32_t hw, int32_t c, int32_t ld, const float* ab,
                          int32_t ab_c, int32_t silu, float out_mul, void* y, int32_t yld, int32_t dtype,
                          void* stream);
/* LayerNorm over the last dim of rows [rows][ld] (first c columns). */
int rdeic_layernorm(const void* x, int32_t rows, int32_t c, int32_t ld, const float* gamma, const float* beta,
                    float eps, void* y, int32_t yld, int32_t dtype, void* stream);

/* ------------------------------------------------------------- attention
 * softmax(Q K^T * scale) V per (batch, head); Q [b][lq][ldq] with head h at columns
 * h*dh..h*dh+dh-1 (same for K/V/O), i.e. the reference's 'b n (h d)' layout.
 * dh in {16, 32, 64}; any lq, lk >= 1. kv_bcast = 1: K/V hold a single batch shared by all
 * `batch` query batches (the one text context of the cross-attention).
 * dh = 512 (bf16, heads = 1, lk % 32 == 0, no kv_bcast): the VAE AttnBlock (model.py:181-205) as a
 * flash kernel, no score matrix in memory. */
int rdeic_attention(const void* q, int32_t ldq, const void* k, int32_t ldk, const void* v, int32_t ldv,
                    void* o, int32_t ldo, int32_t batch, int32_t heads, int32_t lq, int32_t lk, int32_t dh,
                    float scale, int32_t kv_bcast, int32_t dtype, void* stream);
/* materialised-attention helpers (VAE d=512 single-head path in fp32 parity mode): row softmax of
 * s*scale -> p, and batched 2-D transpose. */
int rdeic_softmax_rows(const float* s, int64_t rows, int32_t cols, float scale, void* p, int32_t dtype, void* stream);
int rdeic_transpose(const void* in, int32_t rows, int32_t cols, int32_t ldin, void* out, int32_t ldout,
                    int32_t batch, int64_t in_bs, int64_t out_bs, int32_t dtype, void* stream);

/* ----------------------------------------------------------- elementwise */
/* x * gelu(gate) where x = in[:, :c], gate = in[:, c:2c] (GEGLU, attention.py:49-56) */
int rdeic_geglu(const void* in, int32_t rows, int32_t c, int32_t ldin, void* out, int32_t ldout,
                int32_t dtype, void* stream);
/* dtype / layout conversions between the reference's NCHW fp32 tensors and internal NHWC */
int rdeic_nchw_to_nhwc(const float* in, int32_t n, int32_t c, int32_t h, int32_t w, float mul, float add,
                       void* out, int32_t ld, int32_t dtype, void* stream);
int rdeic_nhwc_to_nchw(const void* in, int32_t n, int32_t c, int32_t h, int32_t w, int32_t ld, float mul,
                       float add, float* out, int32_t dtype, void* stream);
/* generic strided elementwise y = a*x + b*z (+ per-image scalars), used by samplers / q_sample */
int rdeic_axpby(const float* x, const float* z, int32_t n_img, int32_t per_img, const float* a,
                const float* b, float* y, void* stream);
/* sinusoidal timestep embedding [cos(t*f), sin(t*f)] (util.py:161-181); freqs = the model's fp32
 * frequency table exp(-ln(1e4) * arange(dim/2) / (dim/2)) */
int rdeic_timestep_embedding(const int64_t* t, const float* freqs, int32_t n, int32_t dim, float* out, void* stream);
/* relay-DDIM eta=0 update (ddim_sampler_relay.py:215-229) with host-precomputed fp32 scalars */
int rdeic_ddim_step(const float* x, const float* e, int64_t count, float c_sq1m, float c_sqa, float c_sqap,
                    float c_dir, float* xp, float* x0, void* stream);
/* classifier-free guidance combine out = e_uncond + scale * (e_cond - e_uncond), fp32, the reference's op
 * order (ddim_sampler_relay.py:188-192 p_sample_ddim; spaced_sampler_relay.py:277-283 predict_noise) */
int rdeic_cfg_combine(const float* e_cond, const float* e_uncond, int64_t count, float scale, float* out,
                      void* stream);
/* relay spaced (DDPM) update (spaced_sampler_relay.py:270-275 _predict_xstart_from_eps, :154-170
 * q_posterior_mean_variance, :378-383 x_prev): pred_x0 = a*x - b*e, mean = c1*pred_x0 + c2*x,
 * xp = mean + s*noise (s = nonzero_mask * sqrt(model_variance)); fp32 scalars from the host's
 * float64 schedule; noise may be NULL only when s == 0; x0 (pred_x0 out) may be NULL. */
int rdeic_spaced_step(const float* x, const float* e, const float* noise, int64_t count, float a, float b, float c1,
                      float c2, float s, float* xp, float* x0, void* stream);
/* SiLU in place / copy (fp32), for embedding MLP inputs */
int rdeic_silu_f32(const float* x, float* y, int64_t count, void* stream);
/* image u8 HWC <-> model tensors (inference.py:51-52, 85-87). u8 -> NHWC writes x*2-1 into channels
 * 0..2 and, when ld <= 16, zeros into channels 3..ld-1 (a zero-padded conv input). */
int rdeic_image_u8_to_nhwc(const uint8_t* img, int32_t n, int32_t h, int32_t w, void* out, int32_t ld,
                           int32_t dtype, void* stream);
int rdeic_nhwc_to_image_u8(const void* x, int32_t n, int32_t h, int32_t w, int32_t ld, uint8_t* img,
                           int32_t dtype, void* stream);
/* per-image MSE of two uint8 image batches (n images of per_img bytes) -> out[n] (PSNR metric) */
int rdeic_image_mse(const uint8_t* a, const uint8_t* b, int32_t n, int64_t per_img, float* out, void* stream);
/* counter-based synthetic weights: out[i] = ((splitmix64(seed + i) >> 40) - 2^23) * scale + offset */
int rdeic_fill_uniform(float* out, int64_t count, uint64_t seed, float scale, float offset, void* stream);
/* fp32 -> packed conv weight [cout][wld] (zero tail), from torch layout [cout][cin][kh][kw] */
int rdeic_pack_conv_weight(const float* w, int32_t cout, int32_t cin, int32_t kh, int32_t kw, void* out,
                           int32_t wld, int32_t dtype, void* stream);
int rdeic_cast(const void* in, int32_t in_dtype, void* out, int32_t out_dtype, int64_t count, void* stream);

/* ---------------------------------------------------- entropy-model kernels
 * Checkerboard stage of slice `sl` (phase 0 = anchor, 1 = non-anchor) over a [n][hy][wy] latent.
 * params: [pix][pld] with scales at channel 0..c-1 and means at c..2c-1 (chunk(2,1)).
 * Encode: y -> symbols/indexes written per image at sym + img*img_stride + off + (ch*hy + r)*(wy/2) + j
 * and yhat (= sym + mean) scattered to yhat[pix][yld] (+ anchor-only copy when anchor_out != NULL).
 * scale_table: the 64 GaussianConditional levels; lower bound 0.11 (compressai default).
 * sym / idx (and rdeic_ckbd_indexes' idx, rdeic_ckbd_dequant's sym) may be device memory or pinned
 * host memory (hipHostMalloc / torch pin_memory: device-addressable), so the coder round trips need
 * no copy launches; the caller orders host access with an event after the kernel. */
int rdeic_ckbd_encode(const void* y, int32_t yld, const void* params, int32_t pld, int32_t n, int32_t hy,
                      int32_t wy, int32_t c, int32_t phase, const float* scale_table, int32_t levels,
                      float scale_bound, int32_t* sym, int32_t* idx, int64_t img_stride, int64_t off,
                      void* yhat, int32_t yhld, void* anchor_out, int32_t ald, int32_t dtype, void* stream);
/* Index-only pass for decode (build_indexes on the squeezed scales). */
int rdeic_ckbd_indexes(const void* params, int32_t pld, int32_t n, int32_t hy, int32_t wy, int32_t c,
                       int32_t phase, const float* scale_table, int32_t levels, float scale_bound,
                       int32_t* idx, int64_t img_stride, int64_t off, int32_t dtype, void* stream);
/* Decode-side dequantise: yhat = sym + mean scattered like rdeic_ckbd_encode. */
int rdeic_ckbd_dequant(const int32_t* sym, const void* params, int32_t pld, int32_t n, int32_t hy,
                       int32_t wy, int32_t c, int32_t phase, int64_t img_stride, int64_t off, void* yhat,
                       int32_t yhld, void* anchor_out, int32_t ald, int32_t dtype, void* stream);
/* Vector quantiser nearest code (compression_modules.py:309-331): given dot[r][j] = z_r.e_j (from
 * rdeic_conv2d), zn = ||z_r||^2, en = ||e_j||^2: idx[r] = first argmin_j (zn[r] + en[j]) - 2 dot[r][j]. */
int rdeic_vq_argmin(const float* dot, const float* zn, const float* en, int32_t rows, int32_t ncode, int32_t* idx,
                    void* stream);
/* out[r] = table[idx[r]] (fp32 table, output dtype `dtype`): get_codebook_entry / z_q gather */
int rdeic_gather_rows(const float* table, int32_t ld_table, const int32_t* idx, int32_t rows, int32_t dim,
                      void* out, int32_t ld_out, int32_t dtype, void* stream);
int rdeic_row_sqnorm(const void* x, int32_t rows, int32_t dim, int32_t ld, float* out, int32_t dtype,
                     void* stream);

/* ------------------------------------------------------------ image quality
 * SSIM / MS-SSIM of uint8 RGB image pairs [n][h][w][3] (the reference's pyiqa "ssim" / "ms_ssim"
 * with test_y_channel, experiments/run_robustness.py:70-83; restated, parity unpinned): YIQ luma
 * rounded to integers, 11x11 Gaussian (sigma 1.5) 'valid' windows, data range 255, `levels` scales
 * with 2x2 average pooling between them. out[img][level][2] = (mean ssim, mean relu'd cs) of each
 * level; SSIM = out[.][0][0], MS-SSIM = prod_{l<4} cs_l^w_l * ssim_4^w_4 (host).
 * ws: rdeic_image_ssim_ws_floats(n, h, w, levels) floats of device scratch. */
size_t rdeic_image_ssim_ws_floats(int32_t n, int32_t h, int32_t w, int32_t levels);
int rdeic_image_ssim(const uint8_t* a, const uint8_t* b, int32_t n, int32_t h, int32_t w, int32_t levels, float* ws,
                     size_t ws_floats, float* out, void* stream);

/* ------------------------------------------------------------ host coders
 * Gaussian-conditional tables (compressai 1.2.4 GaussianConditional.update, precision 16).
 * pmf: [levels][pmf_ld] float32 pmf rows of length pmf_len[i] followed by the tail mass
 * (computed by the caller exactly as compressai does, in float32); out cdf [levels][cdf_ld]. */
int rdeic_pmf_to_quantized_cdf(const float* pmf, int32_t n, int32_t precision, uint32_t* cdf_out);
int rdeic_build_gaussian_tables(const float* pmf, const int32_t* pmf_len, int32_t levels, int32_t pmf_ld,
                                int32_t* cdf, int32_t cdf_ld, int32_t* cdf_len, void* reserved);

/* rANS (compressai BufferedRansEncoder::encode_with_indexes + flush, rans64, 16-bit, 4-bit bypass). */
int rdeic_rans_encode(const int32_t* sym, const int32_t* idx, size_t n, const int32_t* cdf, int32_t cdf_ld,
                      const int32_t* cdf_len, const int32_t* offset, int32_t levels, uint8_t* out, size_t cap,
                      size_t* out_len);
/* Batched: `count` independent streams (one per image) encoded on host threads. */
int rdeic_rans_encode_batch(int32_t count, const int32_t* sym, const int32_t* idx, size_t n_per,
                            size_t stride, const int32_t* cdf, int32_t cdf_ld, const int32_t* cdf_len,
                            const int32_t* offset, int32_t levels, uint8_t* out, size_t cap_per,
                            size_t* out_len, int32_t threads);
/* The same streams from precomputed per-(row, value) encoder symbols: start, freq and the exact
 * reciprocal of freq (Alverson; ryg_rans Rans64EncSymbolInit), so the flush is ONE reverse pass
 * over the symbols with no 64-bit division and no intermediate symbol list. Tables are built once
 * per GaussianConditional table set, are immutable and are shared by all threads (NULL on a bad
 * table). rdeic_rans_encode_batch_t writes the bytes rdeic_rans_encode_batch writes;
 * rdeic_rans_enc_quotient exposes one reciprocal division (floor(x / freq)) for tests. */
void* rdeic_rans_enc_tables_create(const int32_t* cdf, int32_t cdf_ld, const int32_t* cdf_len,
                                   const int32_t* offset, int32_t levels);
void rdeic_rans_enc_tables_destroy(void* tables);
int rdeic_rans_encode_batch_t(const void* tables, int32_t count, const int32_t* sym, const int32_t* idx,
                              size_t n_per, size_t stride, uint8_t* out, size_t cap_per, size_t* out_len,
                              int32_t threads);
int rdeic_rans_enc_quotient(const void* tables, int32_t row, int32_t value, uint64_t x, uint64_t* q);
void* rdeic_rans_dec_open(const uint8_t* data, size_t len);
int rdeic_rans_decode(void* handle, const int32_t* idx, size_t n, const int32_t* cdf, int32_t cdf_ld,
                      const int32_t* cdf_len, const int32_t* offset, int32_t levels, int32_t* out);
/* Batched decode step: handles[i] decodes n_per symbols (idx + i*stride) into out + i*stride. */
int rdeic_rans_decode_batch(int32_t count, void** handles, const int32_t* idx, size_t n_per, size_t stride,
                            const int32_t* cdf, int32_t cdf_ld, const int32_t* cdf_len, const int32_t* offset,
                            int32_t levels, int32_t* out, int32_t threads);
void rdeic_rans_dec_close(void* handle);

/* torchac 0.9.3-compatible binary arithmetic coder for a shared int16 CDF row of length lp
 * (cdf_int as produced by torchac's _convert_to_int_and_normalize; read as uint16). */
int rdeic_ac_encode(const int16_t* sym, size_t n, const int16_t* cdf_row, int32_t lp, uint8_t* out,
                    size_t cap, size_t* out_len);
int rdeic_ac_decode(const uint8_t* data, size_t len, size_t n, const int16_t* cdf_row, int32_t lp,
                    int16_t* out);
/* The uniform hyper-latent CDF of utils/ckbd.py:117-128 after torchac's int conversion. */
int rdeic_ac_uniform_cdf(int32_t codebook_size, int16_t* cdf_row);

/* --------------------------------------------------------- launch profiler
 * The conv / attention / GroupNorm launchers bracket their kernels with HIP events on the
 * launch stream while profiling is on (a preallocated ring of `capacity` event pairs, reused;
 * launches beyond it are not recorded). Every event pair is a pair of queue markers that costs
 * GPU time, so launches of at least 50 GFLOP (conv / attention) or 64 MB (GroupNorm) are always
 * timed and the smaller ones in a 1-in-`every` sample (hashed on the per-kind launch counter, so
 * it does not alias with the per-step launch sequence), each sampled launch weighted by `every`.
 * rdeic_prof_read returns, for one kind, the weighted estimates of the launch count, the
 * algorithmic work (FLOPs for conv / attention, bytes for GroupNorm) and the event-timed ms
 * (it synchronizes on the recorded events). rdeic_prof_stop returns the slots used. */
#define RDEIC_PROF_CONV 0        /* rdeic_conv2d / _tile / _splitk (incl. batched GEMMs): 2*M*N*K FLOPs */
#define RDEIC_PROF_ATTN 1        /* rdeic_attention, head dim >= 64: 4*B*H*Lq*Lk*dh FLOPs */
#define RDEIC_PROF_ATTN_SMALL 2  /* rdeic_attention, head dim < 64 */
#define RDEIC_PROF_GN_STATS 3    /* rdeic_groupnorm_stats: bytes read */
#define RDEIC_PROF_GN_APPLY 4    /* rdeic_groupnorm_apply: bytes read + written */
#define RDEIC_PROF_GEMM 5        /* rdeic_gemm_strided (training backward / attention): 2*M*N*K*batch FLOPs */
#define RDEIC_PROF_ATTN_D512 6   /* rdeic_attention, head dim 512 (VAE AttnBlock flash kernel): 4*B*Lq*Lk*512 FLOPs */
#define RDEIC_PROF_CONV_BYTES 7  /* every conv launch (not sampled, no events): algorithmic HBM bytes — input
                                    (each element once), packed weight, output, residual — ms reads 0 */
int rdeic_prof_start(int32_t capacity, int32_t every);
/* Per-shape totals of one kind since rdeic_prof_start: up to cap distinct launch-shape keys (attention: dh << 48 |
 * lq << 32 | lk << 16 | batch x heads, 16 bits each) with their weighted launches, work and event ms; returns the
 * number written (synchronizes). */
int rdeic_prof_read_keys(int32_t kind, int64_t* keys, int64_t* launches, double* work, double* ms, int32_t cap);
/* Launch counters (always on, one relaxed atomic add per launch): which kernel a dispatcher chose,
 * so tests can assert that a fused path actually ran (e.g. the halo conv, not its fallback). */
#define RDEIC_COUNT_HALO_CONV 0    /* conv3x3_halo_kernel (GroupNorm-input 3x3 convs, VAE geometry) */
#define RDEIC_COUNT_GN_APPLY 1     /* rdeic_groupnorm_apply kernels */
#define RDEIC_COUNT_LAYERNORM 2    /* rdeic_layernorm kernels */
#define RDEIC_COUNT_HALO_SMALL 3   /* the small-image halo conv (UNet / control ResBlocks) */
#define RDEIC_COUNT_LN_FUSED 4     /* rdeic_layernorm_rowstats (LayerNorm folded into the next linear) */
#define RDEIC_COUNT_SPLITK 5       /* rdeic_conv2d_splitk launches that ran split (partial pass + reduce) */
#define RDEIC_COUNT_EDGE 6         /* the VAE edge convs (conv_edge.hip: conv_in from 8 channels, norm -> SiLU -> conv to <= 16) */
#define RDEIC_COUNT_GN_PARTS_APPLY 7 /* rdeic_groupnorm_parts_apply (finalize + apply in one launch) */
#define RDEIC_COUNT_KINDS 8
int64_t rdeic_launch_count(int32_t kind);
/* Per-row LayerNorm statistics (attention.py:273-285, torch.nn.LayerNorm: biased variance, eps) of
 * bf16 rows x[rows][c] (pixel stride ld): ms[2 r] = mean, ms[2 r + 1] = 1 / sqrt(var + eps), two-pass
 * in registers. The folded linear (rdeic_conv_desc.ln_rows) consumes them; replaces rdeic_layernorm's
 * normalised tensor (never written). c % 8 == 0, c <= 2048. */
int rdeic_layernorm_rowstats(const void* x, int32_t rows, int32_t c, int32_t ld, float eps, float* ms,
                             void* stream);
int rdeic_launch_count_reset(void);
int rdeic_prof_stop(void);
int rdeic_prof_read(int32_t kind, int64_t* launches, double* work, double* ms);

/* ------------------------------------------------ adapter fine-tune step (config 5, train.hip)
 * Replace the autograd backward of the modules the reference's fine-tune trains or back-propagates
 * through (model/rdeic.py:763-881 configure_optimizers / p_losses, model/compression.py:52-149,
 * model/compression_modules.py:228-307, ldm/modules/diffusionmodules/openaimodel.py:162-274,
 * ldm/modules/attention.py:49-56,153-203,255-285) and torch.optim.AdamW.
 *
 * Strided batched GEMM on MFMA: C[z](i,j) = alpha * sum_kk A[z](i,kk) B[z](kk,j) + beta * C[z](i,j),
 * A(i,kk) = a[i*a_sm + kk*a_sk], B(kk,j) = b[kk*b_sk + j*b_sn], C(i,j) = c[i*c_sm + j]; batch
 * z = z1*nb2 + z2 adds z1*x_bs1 + z2*x_bs2 to every operand. ksplit > 0: z1 selects the k-range
 * [z1*ksplit, (z1+1)*ksplit) instead (A/B bs1 unused; C plane z1*c_bs1), for split-K weight
 * gradients. dtype 0 fp32 / 1 bf16 inputs; c_f32 = 1 writes fp32 C. rsum (optional, NULL = off):
 * also the row sums of A over this launch's k range, fp32 [m] at rsum + z1*rsum_bs (the bias
 * gradient of a weight-gradient GEMM, whose A = dy^T; batch z2 must be 0). */
typedef struct rdeic_gemm_desc {
  const void* a;
  int64_t a_bs1, a_bs2, a_sm, a_sk;
  const void* b;
  int64_t b_bs1, b_bs2, b_sk, b_sn;
  void* c;
  int64_t c_bs1, c_bs2, c_sm;
  int32_t batch, nb2, m, n, k, ksplit, dtype, c_f32;
  float alpha, beta;
  float* rsum;
  int64_t rsum_bs;
} rdeic_gemm_desc;
int rdeic_gemm_strided(const rdeic_gemm_desc* d, void* stream);
/* conv input gradient = the forward conv of dy with this flipped / transposed packing of the fp32
 * torch-layout weight [cout][cin][kh][kw] ([cin][wld], K order (ky, kx, co)) and pad kh-1-pad;
 * stride 2: dy zero-inserted first; nearest-up input: the 2x2 sums of the gradient (sum_pool2);
 * PixelShuffle(2) output: pixel_unshuffle2 of the gradient first. h, w are the small grid. */
int rdeic_pack_conv_weight_dgrad(const float* w, int32_t cout, int32_t cin, int32_t kh, int32_t kw, void* out,
                                 int32_t wld, int32_t to_bf16, void* stream);
/* Every trainable layer's packing in one launch (the fine-tune step repacks its trainable weights
 * after each AdamW update): job j packs w into out as rdeic_pack_conv_weight (mode 0, [cout][wld])
 * or rdeic_pack_conv_weight_dgrad (mode 1, [cin][wld]); `start` is the job's first output ROW in the
 * concatenation of all jobs' rows (ascending, start[0] = 0), total = the number of rows. One
 * workgroup per row stages the row's sources in LDS: row_floats = the largest kh*kw*cin (mode 0) /
 * kh*kw*cout (mode 1) over the jobs, at most 36864. jobs points to DEVICE memory. to_bf16 applies
 * to every job. */
typedef struct rdeic_pack_job {
  const float* w;
  void* out;
  int64_t start;
  int32_t cout, cin, kh, kw, wld, mode;
} rdeic_pack_job;
int rdeic_pack_batch(const rdeic_pack_job* jobs, int32_t njobs, int64_t total, int32_t row_floats, int32_t to_bf16,
                     void* stream);
int rdeic_zero_insert2(const void* src, int32_t n, int32_t h, int32_t w, int32_t c, int32_t ld, void* dst,
                       int32_t dst_ld, int32_t dtype, void* stream);
int rdeic_sum_pool2(const void* src, int32_t n, int32_t h, int32_t w, int32_t c, int32_t ld, void* dst,
                    int32_t dst_ld, int32_t dtype, void* stream);
int rdeic_pixel_unshuffle2(const void* src, int32_t n, int32_t h, int32_t w, int32_t c, int32_t ld, void* dst,
                           int32_t dst_ld, int32_t dtype, void* stream);
/* weight gradient: im2col rows [p][(ky,kx,ci)] of the conv input, the split-K GEMM dy^T . cols, then
 * the sum of the split planes written (or added) in torch layout [cout][cin][kh][kw]; db (optional):
 * the bias gradient, the split-order sum of the GEMM's row-sum planes rpart [splits][cout] (same
 * accumulate mode) */
int rdeic_im2col(const void* x, int32_t n, int32_t h, int32_t w, int32_t c, int32_t ld, int32_t kh, int32_t kw,
                 int32_t stride, int32_t pad_t, int32_t pad_l, int32_t ho, int32_t wo, int32_t up2, void* out,
                 int64_t out_ld, int32_t dtype, void* stream);
int rdeic_wgrad_finalize(const float* part, int32_t splits, int32_t cout, int32_t cin, int32_t kh, int32_t kw,
                         float* dw, int32_t accumulate, const float* rpart, float* db, void* stream);
/* out[g][c] (+)= sum of the rows of group g (rows split into `groups` equal runs): bias / emb grads */
size_t rdeic_col_sum_ws_floats(int64_t rows, int32_t c, int32_t groups);
int rdeic_col_sum(const void* x, int64_t rows, int32_t c, int32_t ld, int32_t groups, float* out, int32_t accumulate,
                  float* ws, size_t ws_floats, int32_t dtype, void* stream);
/* act: 1 leaky (slope), 2 exact GELU, 3 SiLU. fwd: out = act(z) (+ res); bwd: dz = dy * act'(z) */
int rdeic_act_fwd(const void* z, int64_t rows, int32_t c, int32_t ldz, const void* res, int32_t ldr, int32_t act,
                  float slope, void* out, int32_t ldo, int32_t dtype, void* stream);
int rdeic_act_bwd(const void* dy, int32_t ldy, const void* z, int32_t ldz, int64_t rows, int32_t c, int32_t act,
                  float slope, void* dz, int32_t lddz, int32_t dtype, void* stream);
/* GroupNorm training forward: mean / rstd per (image, group) -> mr [n][g][2] and the affine
 * ab [n][c][2] (apply with rdeic_groupnorm_apply); backward (+ SiLU when silu) -> dx, dgamma,
 * dbeta (null: not wanted). ws: rdeic_gn_train_ws_doubles; coef: [n][g][2] floats. */
size_t rdeic_gn_train_ws_doubles(int32_t n, int32_t hw, int32_t c);
int rdeic_gn_train_fwd(const void* x, int32_t ldx, int32_t n, int32_t hw, int32_t c, int32_t groups, float eps,
                       const float* gamma, const float* beta, float* mr, float* ab, double* ws, int32_t dtype,
                       void* stream);
int rdeic_gn_train_bwd(const void* x, int32_t ldx, const void* dy, int32_t ldy, int32_t n, int32_t hw, int32_t c,
                       int32_t groups, const float* mr, const float* gamma, const float* beta, int32_t silu, void* dx,
                       int32_t lddx, float* dgamma, float* dbeta, int32_t accumulate, double* ws, float* coef,
                       int32_t dtype, void* stream);
/* the same with a second gradient of x added (dres [n*hw][ldr], null: none): dx = round(round(dx_gn) + dres), what
 * autograd's sum of the two gradient tensors gives (the residual path of a block whose input feeds this norm) */
int rdeic_gn_train_bwd_res(const void* x, int32_t ldx, const void* dy, int32_t ldy, int32_t n, int32_t hw, int32_t c,
                           int32_t groups, const float* mr, const float* gamma, const float* beta, int32_t silu,
                           const void* dres, int32_t ldr, void* dx, int32_t lddx, float* dgamma, float* dbeta,
                           int32_t accumulate, double* ws, float* coef, int32_t dtype, void* stream);
/* LayerNorm backward (statistics recomputed); dgamma / dbeta optional (ws then required) */
size_t rdeic_layernorm_bwd_ws_floats(int64_t rows, int32_t c);
int rdeic_layernorm_bwd(const void* x, int32_t ldx, int64_t rows, int32_t c, const float* gamma, float eps,
                        const void* dy, int32_t ldy, void* dx, int32_t lddx, float* dgamma, float* dbeta,
                        int32_t accumulate, float* ws, size_t ws_floats, int32_t dtype, void* stream);
/* ... with a second gradient of x added (dres [rows][ldr], null: none), as rdeic_gn_train_bwd_res */
int rdeic_layernorm_bwd_res(const void* x, int32_t ldx, int64_t rows, int32_t c, const float* gamma, float eps,
                            const void* dy, int32_t ldy, const void* dres, int32_t ldr, void* dx, int32_t lddx,
                            float* dgamma, float* dbeta, int32_t accumulate, float* ws, size_t ws_floats,
                            int32_t dtype, void* stream);
/* ds = p * (dp - rowsum(p * dp)) * scale  (p [rows][cols] of rdeic_softmax_rows, dp fp32) */
int rdeic_softmax_bwd_rows(const void* p, const float* dp, int64_t rows, int32_t cols, float scale, void* ds,
                           int32_t dtype, void* stream);
/* GEGLU backward: x = [value | gate] [rows][2c], dy [rows][c] -> dx [rows][2c] */
int rdeic_geglu_bwd(const void* x, int32_t ldx, int64_t rows, int32_t c, const void* dy, int32_t ldy, void* dx,
                    int32_t lddx, int32_t dtype, void* stream);
/* checkerboard entropy slice in training mode (compression.py:80-139; compressai 1.2.4
 * GaussianConditional noise-mode likelihood, LowerBound(0.11) scale, LowerBound(1e-9) likelihood,
 * quantize_ste). Params [scales (c) | means (c)] per pixel; anchors at (row + col) odd.
 *   anchor:   out = anchor ? round(y - mu_a) + mu_a : 0
 *   lik:      out2 = (sum ln lik(y + noise), sum ln lik(round(y - mu) + mu)); nonanchor_hat likewise
 *   lik_bwd:  from dL/d(sum ln lik) (device scalar) and d nonanchor_hat -> dy, dpa, dpn */
int rdeic_ckbd_train_anchor(const void* y, int32_t ldy, const void* pa, int32_t ldpa, int32_t n, int32_t h, int32_t w,
                            int32_t c, void* out, int32_t ldo, int32_t dtype, void* stream);
/* out = x at anchor (which = 1) / non-anchor (which = 0) positions, 0 elsewhere */
int rdeic_ckbd_mask(const void* x, int32_t ldx, int32_t n, int32_t h, int32_t w, int32_t c, int32_t which, void* out,
                    int32_t ldo, int32_t dtype, void* stream);
size_t rdeic_ckbd_train_ws_doubles(int32_t n, int32_t h, int32_t w, int32_t c);
int rdeic_ckbd_train_lik(const void* y, int32_t ldy, const void* pa, int32_t ldpa, const void* pn, int32_t ldpn,
                         const float* noise, int32_t n, int32_t h, int32_t w, int32_t c, void* nonanchor_hat,
                         int32_t ldo, double* ws, float* out2, int32_t dtype, void* stream);
int rdeic_ckbd_train_lik_bwd(const void* y, int32_t ldy, const void* pa, int32_t ldpa, const void* pn, int32_t ldpn,
                             const float* noise, int32_t n, int32_t h, int32_t w, int32_t c, const float* g_sum,
                             const void* d_nonanchor, int32_t ldd, void* dy, int32_t lddy, void* dpa, int32_t lddpa,
                             void* dpn, int32_t lddpn, int32_t dtype, void* stream);
/* VectorQuantiser.forward (training, anchor 'closest', contrastive loss) per code e, from
 * dot = z . E^T [P][K], |z_p|^2, |E_e|^2 and the nearest-code indexes: re-initialises E and
 * embed_prob in place, writes code_out [K][2] (CE_e, commitment sq-dist), dE_unit [K][D]
 * (d emb_loss / dE for upstream gradient 1) and loss3 = (emb_loss, mse, mean CE). P <= 4096,
 * D <= 512. vq_z_grad: dz = dzq + g_loss * coef * (z - zq). scale_dev: y (+)= s[0] * x. */
int rdeic_vq_train(const float* dot, const float* zn, const float* en, const float* z, const int32_t* idx, int32_t P,
                   int32_t K, int32_t D, float* E, float* embed_prob, float beta, float decay, float temp,
                   float* code_out, float* dE_unit, float* loss3, void* stream);
int rdeic_vq_z_grad(const float* z, const float* zq, const void* dzq, int64_t count, const float* g_loss, float coef,
                    void* dz, int32_t dtype, void* stream);
int rdeic_scale_dev(const float* x, int64_t count, const float* s, float* y, int32_t accumulate, void* stream);
/* torch.optim.AdamW (decoupled weight decay) over flat fp32 buffers, step >= 1 */
int rdeic_adamw(float* p, const float* g, float* m, float* v, int64_t count, float lr, float beta1, float beta2,
                float eps, float weight_decay, int32_t step, void* stream);
/* the same update with step_scalars = device [-lr / (1 - beta1^step), sqrt(1 - beta2^step)] (graph replay) */
int rdeic_adamw_dev(float* p, const float* g, float* m, float* v, int64_t count, float lr, float beta1, float beta2,
                    float eps, float weight_decay, const float* step_scalars, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* RDEIC_HIP_H */
