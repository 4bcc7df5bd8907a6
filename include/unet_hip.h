/*
 * unet_hip.h -- C-ABI of libunet_hip.so, the MI355X (gfx950) implementation of
 * the valid-convolution U-Net training / inference hot path of
 * SaurabhIndi/unet-segmentation (reference snapshot 2025-07-25).
 *
 * The reference has no FFI: its boundary is the nn.Module API
 *   models/unet_model.py:66   UNet(n_channels, n_classes, bilinear=False)
 *   models/unet_model.py:105  UNet.forward(x) -> logits (N, n_classes, H-184, W-184)
 *   utils/losses.py:29        WeightedCrossEntropyLoss.forward(inputs, targets, weight_maps)
 *   scripts/train.py:97,131   optim.SGD(lr=1e-4, momentum=0.99).step()
 * These entry points are what a Python (ctypes) binding of that boundary calls;
 * unet-segmentation_amd/unet_amd/_lib.py is that binding.
 *
 * Conventions
 *  - Every pointer is a DEVICE pointer unless the name says host_.  Buffers are
 *    owned by the caller (PyTorch caching allocator); the library never
 *    allocates device memory.
 *  - Activations are NHWC float32 ("_nhwc"); the network input x and the
 *    logits use the reference's NCHW layout.
 *  - Parameter tables are host arrays of device pointers in the reference
 *    state_dict order (136 entries incl. BN buffers; 82 gradient entries in
 *    named_parameters order).  Shapes are PyTorch's (Conv2d OIHW,
 *    ConvTranspose2d IOHW).
 *  - stream is a hipStream_t (torch.cuda.current_stream().cuda_stream).
 *  - Return 0 on success, a negative errno-style code on bad arguments
 *    (-EINVAL) or a HIP launch failure (-EIO); never throws across the ABI.
 *    unet_last_error() returns a static message for the last failure.
 */
#ifndef UNET_HIP_H
#define UNET_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* unet_stream_t; /* hipStream_t */

/* "unet_hip <ver> gfx950 ... src <hash>": <hash> = the first 16 hex digits of
 * sha256 over the library's sources (csrc/Makefile SRC_HASH), so a run's record
 * shows which sources the loaded .so was built from. */
const char* unet_version(void);
const char* unet_last_error(void);

/* ------------------------------------------------------------------------
 * Whole-network plan: one plan per (N, C, H, W, n_classes).  Replaces the
 * body of UNet.forward (models/unet_model.py:105-146) and autograd's backward
 * through it.
 * ---------------------------------------------------------------------- */
typedef struct unet_plan unet_plan;

/* Create a plan; returns NULL (and sets unet_last_error) for sizes the valid
 * U-Net cannot take (models/unet_model.py:189: out = in - 184 for clean sizes)
 * and for c_in or n_classes outside 1..4096 (the reference's
 * UNet(n_channels, n_classes), models/unet_model.py:66-85, takes any counts;
 * the bound only keeps the per-plan buffers in reason: the first conv stages
 * its input channels in chunks of 16, the head / loss run register-blocked up
 * to 32 classes and with a run-time class loop above).
 * unet_plan_create() is unet_plan_create_ex(..., UNET_PREC_FP32). */
unet_plan* unet_plan_create(int n, int c_in, int h, int w, int n_classes);

/* Arithmetic of the implicit-GEMM convolutions (the 17 3x3 convs after the
 * first, the 4 ConvTranspose2d, their input and weight gradients):
 *  UNET_PREC_FP32  fp32 operands, exact fp32 MFMA (configs C1/C2, the parity
 *                  configuration);
 *  UNET_PREC_BF16  both operands rounded to bf16 (RNE) when staged, fp32
 *                  accumulation (v_mfma_f32_32x32x16_bf16): the "bf16-in /
 *                  fp32-acc" of configs C3/C5, what torch.autocast(bfloat16)
 *                  asks of the reference's convolutions;
 *  UNET_PREC_BF16X3 fp32-accurate GEMMs on the bf16 matrix cores: each fp32
 *                  operand is split v = hi + lo (hi = bf16(v), lo = bf16(v -
 *                  hi), |v - hi - lo| <= 2^-16 |v|) and a product is taken as
 *                  hi*hi' + hi*lo' + lo*hi' (three v_mfma_f32_32x32x16_bf16,
 *                  fp32 accumulation; the dropped lo*lo' is <= 2^-16 of the
 *                  product).  Storage as in UNET_PREC_FP32; tested against the
 *                  fp64 oracle at the fp32 tolerances.
 * Everything else -- the first conv (any Ci), the 1x1 head, BatchNorm, the
 * loss, gradients and the optimizer -- is fp32 in all three; UNET_PREC_BF16
 * plans also store the GEMM-only tensors and the raw conv outputs in bf16. */
enum { UNET_PREC_FP32 = 0, UNET_PREC_BF16 = 1, UNET_PREC_BF16X3 = 2 };
unet_plan* unet_plan_create_ex(int n, int c_in, int h, int w, int n_classes, int precision);
int unet_plan_precision(const unet_plan* p);
void unet_plan_destroy(unet_plan* p);
/* Output spatial size and the workspace the caller must provide.
 * unet_plan_workspace_bytes: a forward followed by unet_plan_backward.
 * unet_plan_forward_workspace_bytes: a forward that no backward follows (eval
 * mode -- scripts/predict.py -- or a train-mode forward under torch.no_grad);
 * a prefix of the full layout, about 1/3 of it (the gradient buffers are left
 * out).  Running unet_plan_backward on such a workspace is undefined. */
int unet_plan_out_hw(const unet_plan* p, int* out_h, int* out_w);
size_t unet_plan_workspace_bytes(const unet_plan* p);
size_t unet_plan_forward_workspace_bytes(const unet_plan* p);
int unet_plan_num_params(const unet_plan* p);  /* 136 (state_dict entries) */
int unet_plan_num_grads(const unet_plan* p);   /* 82 */

/* Forward.  train=1: BatchNorm uses batch statistics and updates the running
 * buffers in place (momentum 0.1, unbiased var, num_batches_tracked += 1);
 * train=0: running statistics (scripts/predict.py:70 model.eval()).
 * host_params[136]: device pointers of the state_dict tensors.
 * x_nchw: (N, C, H, W) float32 contiguous.  logits_nchw: (N, K, Ho, Wo).
 * workspace: unet_plan_workspace_bytes() bytes, 256-B aligned; it holds the
 * activations the backward needs, so keep it alive until unet_plan_backward. */
int unet_plan_forward(unet_plan* p, void* const* host_params, const float* x_nchw,
                      float* logits_nchw, void* workspace, int train, unet_stream_t stream);

/* Backward of the whole network for dlogits (N, K, Ho, Wo).  Writes (does not
 * accumulate) the 82 parameter gradients to host_grads[].  Segments let a
 * data-parallel caller all-reduce finished gradients while the rest runs:
 * segment s in [seg_begin, seg_end) of unet_plan_num_segments(); the full
 * backward is (0, num_segments).  unet_plan_segment_grads() lists, for a
 * segment, which gradient entries are final after it.  x_nchw is the forward
 * input (inc.c0's weight gradient reads it). */
int unet_plan_num_segments(const unet_plan* p);
int unet_plan_segment_grads(const unet_plan* p, int seg, int* first_grad, int* n_grads);
int unet_plan_backward(unet_plan* p, void* const* host_params, void* const* host_grads,
                       const float* x_nchw, const float* dlogits_nchw, void* workspace,
                       int seg_begin, int seg_end, unet_stream_t stream);
/* Gradient of the network input (the reference's x.grad when the input
 * requires grad; models/unet_model.py:105): after the backward segment that
 * holds inc.c0 (segment 8, i.e. a whole backward), materialises inc.c0's
 * BatchNorm-backward output into `scratch` (fp32,
 * unet_plan_input_grad_scratch_bytes) and writes dx (N, C, H, W) fp32.  Same
 * stream as the backward. */
size_t unet_plan_input_grad_scratch_bytes(const unet_plan* p);
int unet_plan_input_grad(unet_plan* p, void* const* params, float* dx, void* workspace, void* scratch,
                         unet_stream_t stream);
/* The same with flags.  UNET_BWD_DEFER_JOIN: the weight gradients of these
 * segments (which run on the plan's side stream beside the input-gradient
 * chain once the plan is tuned) are NOT joined into `stream` on return, so the
 * next segment's input gradients overlap them; a collective over segment s's
 * gradients must first make its stream wait with unet_plan_wait_segment(s),
 * and unet_plan_join() must be called on `stream` before anything reads the
 * gradients or the workspace again (optimizer step, next forward).  This is
 * the data-parallel schedule (unet_amd/train.py): all-reduce bucket s while
 * segment s+1 computes. */
enum { UNET_BWD_DEFER_JOIN = 1 };
int unet_plan_backward_ex(unet_plan* p, void* const* host_params, void* const* host_grads,
                          const float* x_nchw, const float* dlogits_nchw, void* workspace,
                          int seg_begin, int seg_end, int flags, unet_stream_t stream);
int unet_plan_wait_segment(unet_plan* p, int seg, unet_stream_t stream);
int unet_plan_join(unet_plan* p, unet_stream_t stream);

/* Optional per-kernel timing of the next forward/backward: the plan records a
 * hipEvent pair around each launch (class ids below).  unet_plan_timing()
 * returns accumulated milliseconds and algorithmic FLOP/bytes per class. */
enum {
  UNET_KC_CONV_FWD = 0, UNET_KC_CONV_DGRAD = 1, UNET_KC_CONV_WGRAD = 2,
  UNET_KC_STAGE1 = 3,   /* inc.c0 fwd + its BN/ReLU passes (memory-bound) */
  UNET_KC_ELEMWISE = 4, /* BN / pool / head / repack passes */
  UNET_KC_BOTTLENECK = 5, /* overlaps 0-2: the GEMMs of down4.c0, down4.c1,
                             up1.convT, up1.c0 (SURVEY.md §8d's bottleneck set) */
  UNET_KC_COUNT = 6
};
int unet_plan_set_timing(unet_plan* p, int enable);
int unet_plan_timing(const unet_plan* p, double* ms, double* flops, double* bytes, int* launches);
/* MFMA flops the chosen GEMM variants executed per class over the intervals the
 * last unet_plan_timing() call reported: equal to its `flops` (the direct
 * convolution's 2*M*N*K) except where a Winograd variant ran (igemm tiles
 * 70-72/74, wgrad tiles 71/74: 2 * points * tiles * Cin * Cout). */
int unet_plan_timing_mfma_flops(const unet_plan* p, double* mfma_flops);
/* Per GEMM launch site of the last step unet_plan_timing() collected: one line
 * per site, "<layer> <fwd|dgrad|wgrad>\t<ms>\t<direct flops>\t<MFMA flops>".
 * Copies up to cap bytes (NUL-terminated) into buf; returns the size needed. */
size_t unet_plan_timing_sites(const unet_plan* p, char* buf, size_t cap);

/* ------------------------------------------------------------------------
 * Loss: WeightedCrossEntropyLoss (utils/losses.py:29-57) fused fwd+bwd.
 * logits (N, K, H, W) contiguous; targets int64 and weights float32 are read
 * through element strides (the caller's center-cropped views,
 * scripts/train.py:118-126, need no copy).  Writes loss (1 float) and
 * dlogits = w*(softmax - onehot)/(N*H*W) * grad_scale.  ws: 64*8 bytes; on
 * return-to-host ws[1] (double) is 1 if a target was outside [0, k) and not
 * ignore_index -100 (such pixels contribute nothing), ws[2] one such target:
 * torch's nn.CrossEntropyLoss raises for them (utils/losses.py:27), the caller
 * checks the flag at its next synchronisation point.  1 <= k <= 32. */
int unet_wce_fwd_bwd(const float* logits, const int64_t* targets, const float* weights,
                     int n, int k, int h, int w,
                     const int64_t* t_strides /*host, 3*/, const int64_t* w_strides /*host, 3*/,
                     float* loss_out, float* dlogits, float grad_scale, void* ws,
                     unet_stream_t stream);
/* dlogits *= g[0] (the upstream scalar gradient, device), in place. */
int unet_scale_by_device_scalar(float* x, size_t n, const float* g, unet_stream_t stream);
/* y = x * g[0] (y may alias x): the loss backward scales into a fresh tensor so
 * the saved gradient survives a second backward (retain_graph=True). */
int unet_scale_by_device_scalar_out(const float* x, float* y, size_t n, const float* g, unet_stream_t stream);

/* SGD with momentum (torch.optim.SGD, dampening 0, no weight decay), flat,
 * on the gradient g*grad_scale (grad_scale = 1/world after a SUM all-reduce):
 * first_step: buf = g; else buf = momentum*buf + g;  p -= lr*buf.
 * p, g, buf 16-byte aligned.  scripts/train.py:97,131. */
int unet_sgd_momentum(float* p, const float* g, float* buf, size_t n, float lr, float momentum,
                      float grad_scale, int first_step, unet_stream_t stream);

/* Binary IoU of two uint8 masks (utils/metrics.py:6-37), counts on device:
 * out[0] = |pred>0 & gt>0|, out[1] = |pred>0 | gt>0| (uint64). */
int unet_iou_counts(const uint8_t* pred, const uint8_t* gt, size_t n, unsigned long long* out,
                    unet_stream_t stream);
/* mask = (logit1 > logit0) * 255 (scripts/predict.py:85-92), logits NCHW K=2. */
int unet_mask_from_logits(const float* logits, uint8_t* mask, int n, int h, int w,
                          unet_stream_t stream);

/* Elastic-deformation input pipeline: the
 * utils/augmentations.py:4-39 warp and the utils/dataset.py:84-111 steps around
 * it for a batch of n samples (h x w each):
 *   noise  (n, 2, h, w) fp64 uniform [0, 1) -- field 0 drives dx, field 1 dy
 *          (the reference draws them as RandomState(seed).rand(h, w), dx first);
 *   dx|dy = alpha * gaussian_filter(2 noise - 1, sigma, mode="constant")
 *          (truncate 4: radius int(4 sigma + 0.5) <= 160);
 *   image' = map_coordinates(image, (y + dy, x + dx), order=1, mode="reflect"),
 *   label' = same with order=0, both rounded to their integer type;
 *   x_out  (n, h, w) fp32 = uint8(image') / 255   (ToTensor, NCHW with C = 1),
 *   target_out (n, h, w) uint8 = uint8(label') > 0 (the weight map is not
 *          warped, as in the reference);
 *   image_out (optional, may be NULL) = uint8(image').
 * ws >= unet_elastic_ws_bytes(n, h, w), 8-byte aligned. */
size_t unet_elastic_ws_bytes(int n, int h, int w);
int unet_elastic_deform(const uint8_t* image, const uint16_t* labels, int n, int h, int w,
                        const double* noise, double alpha, double sigma, float* x_out,
                        uint8_t* target_out, uint8_t* image_out, void* ws, unet_stream_t stream);

/* Overlap-tile inference (scripts/predict1.py:35-49
 * margin rule): tile t of an nx-wide tile grid has its input origin at
 * ((t / nx) * tile_out - top, (t % nx) * tile_out - left) in the image; a call
 * covers tiles first + b * stride, b < ntiles (stride = world for a round-robin deal).
 * unet_tile_gather: tiles (ntiles, c, tile_in, tile_in) fp32, read from image (c, h, w) with the mirror
 *   padding ("reflect", np.pad semantics incl. pads beyond the image) folded
 *   into the index.
 * unet_tile_scatter: tile logits (ntiles, k, tile_out, tile_out) into the full
 *   logits (k, h, w) (may be NULL) and / or the mask (h, w) uint8 =
 *   255 * (l1 > l0) (k == 2; scripts/predict.py:85-92; may be NULL); output
 *   pixels past the image are dropped. */
int unet_tile_gather(const float* image, int c, int h, int w, int tile_in, int tile_out, int top, int left,
                     int nx, int first, int stride, int ntiles, float* tiles, unet_stream_t stream);
int unet_tile_scatter(const float* tile_logits, int k, int tile_out, int nx, int first, int stride, int ntiles,
                      int h, int w, float* logits, uint8_t* mask, unet_stream_t stream);

/* Loss weight maps (scripts/preprocess_data.py:17-77 with
 * w0, sigma as its :14-15 = 10, 5): per sample of labels (n, h, w) uint16,
 * weights = fp32(wc) + w0 * exp(-(d1 + d2)^2 / (2 (sigma^2 + 1e-8))) where wc =
 * 1 / (class count / h w) of labels > 0 and d1 = d2 = 0 (the reference's
 * min(edt(obj), edt(!obj)) is identically 0).  weights (n, h, w) fp32 (what
 * utils/dataset.py:111 feeds the loss), weights64 (may be NULL) the fp64 map
 * the reference saves.  ws >= unet_weight_map_ws_bytes(n), 8-byte aligned. */
size_t unet_weight_map_ws_bytes(int n);
int unet_weight_map(const uint16_t* labels, int n, int h, int w, double w0, double sigma, float* weights,
                    double* weights64, void* ws, unet_stream_t stream);

/* Post-processing (utils/metrics.py):
 * unet_instance_masks: get_instance_masks (:42-72) for n masks (h, w) uint8
 *   (> 0 = foreground): 8-connected components numbered 1, 2, ... in raster
 *   order of their first pixel (skimage.measure.label(connectivity=2)), those
 *   with fewer than min_size pixels set to 0 without renumbering
 *   (remove_small_objects), uint16 labels out.  n h w < 2^31.
 * unet_rand_index: calculate_rand_index_and_error (:75-139) of two uint16
 *   labelings (h, w): out[0] = Rand index, out[1] = Rand error (fp64, device);
 *   up to 2^24 (gt label, pred label) pairs; synchronises the stream once. */
size_t unet_instance_masks_ws_bytes(int n, int h, int w);
int unet_instance_masks(const uint8_t* mask, int n, int h, int w, int min_size, uint16_t* labels, void* ws,
                        unet_stream_t stream);
size_t unet_rand_index_ws_bytes(int h, int w);
int unet_rand_index(const uint16_t* gt, const uint16_t* pred, int h, int w, double* out, void* ws,
                    unet_stream_t stream);

/* Cell tracking (scripts/track.py:103-275): a tracker
 * consumes the instance labelings of a sequence frame by frame and keeps the
 * lineage (CellTrack :27-36).  Per frame the GPU builds the overlap table of
 * the previous and current objects in one pass (replacing calculate_mask_iou,
 * :73-100, per object pair); the host side runs the reference's control flow:
 * IoU cost matrix (1 - IoU, 1000 where no overlap), linear sum assignment,
 * links with IoU >= iou_track, divisions (an unmatched parent overlapping 2..
 * max_children unmatched objects with IoU >= iou_division), new tracks.
 *   unet_tracker_create(h, w, 0.3, 0.1, 2) = the reference's constants
 *     (:21-24).  NULL for bad sizes.
 *   unet_tracker_add_frame: labels (h, w) uint16 on the device; frame = the
 *     frame number (the reference parses it from mXXX.tif); synchronises the
 *     stream; ws >= unet_tracker_ws_bytes(h, w) bytes, kept for the whole
 *     sequence (it holds the previous frame).
 *   unet_tracker_step_host: the same step from host data -- the current
 *     objects' labels (ascending, > 0), areas, and the overlap counts
 *     inter[i * n_curr + j] with the previous step's objects (NULL on the
 *     first frame).  Host only (no device work).
 *   unet_tracker_tracks: writes up to cap rows (label, start, end, parent) in
 *     the res_track.txt order (start frame, then label; end >= start);
 *     returns the track count.
 * unet_linear_sum_assignment: scipy.optimize.linear_sum_assignment's
 *   minimisation on a row-major nr x nc fp64 cost matrix (host pointers,
 *   min(nr, nc) pairs sorted by row); -EINVAL for NaN / -inf / infeasible. */
typedef struct unet_tracker unet_tracker;
unet_tracker* unet_tracker_create(int h, int w, double iou_track, double iou_division, int max_children);
void unet_tracker_destroy(unet_tracker* t);
size_t unet_tracker_ws_bytes(int h, int w);
int unet_tracker_add_frame(unet_tracker* t, const uint16_t* labels, int frame, void* ws, unet_stream_t stream);
int unet_tracker_step_host(unet_tracker* t, int frame, int n_curr, const int32_t* host_labels,
                           const int64_t* host_areas, const int64_t* host_inter);
int unet_tracker_num_tracks(const unet_tracker* t);
int unet_tracker_tracks(const unet_tracker* t, int32_t* host_out, int cap);
int unet_linear_sum_assignment(long long nr, long long nc, const double* host_cost, int64_t* host_row_ind,
                               int64_t* host_col_ind);

/* Tuning hooks, process-global:
 *  "autotune"      1 (default, or env UNET_AUTOTUNE) = the plan times the
 *                  applicable GEMM variants (tile shape, split-K, wgrad pixel
 *                  split) the first time it meets a GEMM shape and caches the
 *                  fastest per shape; 0 = built-in heuristic only.
 *  "igemm_variant" heuristic override for A/B measurements (-1 = off, 1..9 =
 *                  forced tile shape; 21-26, 31-36, 41-44 bf16 tiles, 63,
 *                  65-68 bf16 halo tiles with LDS-DMA weights; 70-72, 74 fp32
 *                  Winograd: F(2x2,3x3), F(4x4,3x3), fused F(4x4,3x3),
 *                  F(6x6,3x3), plan GEMMs only -- they need the plan's
 *                  scratch); "wgrad_variant"
 *                  (-1 = off, 1 = 64x64 tile, 2..9 = workgroups per CU for the
 *                  pixel split; bf16 GEMMs: 10-14, 20-21 = forced bf16 tile;
 *                  22-23 fp32 halo tiles; 71 / 74 = Winograd F(4x4,3x3) /
 *                  F(6x6,3x3) weight gradient, plan GEMMs only; 1071 / 1074
 *                  the same in slab mode; 100-104 = fp32 pixel-column tile
 *                  0-4 in slab mode; 110-114 / 126-133 bf16 slab modes);
 *  "wino_max"      largest fp32 Winograd output tile the autotuner may pick
 *                  for forward / input-gradient GEMMs (env UNET_WINO_MAX): 6 =
 *                  F(6x6) and below, 4 (default) = F(4x4) / F(2x2), 2 = F(2x2)
 *                  only, 0 = direct GEMMs only; "wino_wgrad_max" (env
 *                  UNET_WINO_WGRAD_MAX, default 6) the same for weight gradients.
 *  "concurrent"    1 (default, or env UNET_CONCURRENT) = a plan's backward
 *                  runs the weight-gradient GEMMs on a side stream beside the
 *                  dX chain (joined before the call returns); 0 = one stream.
 *  "bf16_norm"     1 (or env UNET_BF16_NORM=1; default 0) = UNET_PREC_BF16 plans
 *                  created afterwards write relu(bn(y)) of every layer once
 *                  as a bf16 tensor, the plain operand of its GEMM consumers
 *                  (LDS-DMA staging; tiles 81-84 need it); 0 = consumers apply
 *                  BatchNorm + ReLU while staging.
 *  "bn_fold"       1 (default, or env UNET_BN_FOLD) = eval forwards fold each
 *                  BatchNorm into its conv (weights x gamma / sqrt(var + eps),
 *                  bias x that + beta - mean x that) and store relu(conv') in
 *                  the GEMM epilogue; 0 = consumers apply BN + ReLU on load.
 *  "force_split"   k > 1: every plan igemm runs split-K k (tests), 0 = off.
 *  "force_tile"    id > 0: every plan igemm whose shape admits tile id runs
 *                  it (tests; 1-4, 6-9 register-staged, 11-14 LDS-DMA, 51-54
 *                  fp32 halo, 70-72 / 74 fp32 Winograd, 21-26 / 31-36 / 63-67
 *                  / 81-84 bf16 operands -- only in UNET_PREC_BF16 / _BF16X3
 *                  plans).
 *  "op_precision"  UNET_PREC_* of the per-op GEMM entry points below
 *                  (unet_conv3x3_*, unet_convT2_*); default fp32.
 *  "op_a16"        1 = with op_precision UNET_PREC_BF16, unet_conv3x3_fwd /
 *                  _dgrad store their A operand bf16 first (x rounded before
 *                  the BN+ReLU transform; padded dY bf16), as a bf16 plan
 *                  does -- the configuration the 61-66 tiles (bf16-stored A
 *                  only) run in; 0 (default) = fp32 A.
 *  "deterministic" 1 (or env UNET_DETERMINISTIC=1; default 0) = every weight
 *                  gradient runs a variant without fp32 atomics (slab
 *                  partials summed in a fixed order) and inc.c0's slab
 *                  reduction runs in one pass: plan steps are
 *                  bit-reproducible run to run (see
 *                  unet_nondeterministic_sites).
 *  "bnb_fuse"      1 (default; env UNET_BNB_FUSE) = fp32 plans form the
 *                  BatchNorm-backward dY of a layer whose weight gradient runs
 *                  Winograd F(6x6) in one pass with that weight gradient's dY
 *                  transform (see unet_fused_bnb_sites; read for the workspace
 *                  layout at plan creation); 0 = the two-pass form
 *                  (bit-identical results).
 *  "wgrad_early_u" 1 (default; env UNET_WGRAD_EARLY_U) = the Winograd weight
 *                  gradients' input transform is issued on the side stream
 *                  before the wait for the layer's dY; 0 = after it
 *                  (bit-identical results). */
int unet_set_tuning(const char* key, int value);
/* Text report of the tuned GEMM choices (one line per shape: key, heuristic
 * time, chosen variant and time).  Copies up to len-1 bytes + NUL into buf
 * (buf may be NULL); returns the full report size including the NUL. */
size_t unet_tuning_report(char* buf, size_t len);
/* Forget every tuned choice (the next plan run re-tunes). */
int unet_tuning_reset(void);
/* Slab-mode weight gradients (tuned or forced) that fell back to atomic
 * accumulation because their split partials exceeded the plan's slab; reset
 * != 0 also zeroes the count. */
long long unet_slab_fallbacks(int reset);
/* Deterministic mode (unet_set_tuning("deterministic", 1) or
 * UNET_DETERMINISTIC=1): weight-gradient launch sites that found no
 * atomic-free variant and ran with fp32 atomics; reset != 0 also zeroes the
 * count.  0 after a step means the step is bit-reproducible. */
long long unet_nondeterministic_sites(int reset);
/* Layer backward steps of fp32 plans whose BatchNorm-backward dY was formed by
 * the fused apply + F(6x6) dY-transform pass (unet_set_tuning "bnb_fuse")
 * instead of the standalone apply pass; reset != 0 also zeroes the count.
 * Replaces nothing in the reference: it is a counter of this implementation's
 * schedule (models/unet_model.py:12,16 is the BatchNorm2d it differentiates). */
long long unet_fused_bnb_sites(int reset);
/* Tuning database (cf. MIOpen's perf-db): unet_tuning_save writes every tuned
 * choice as "key<TAB>tile<TAB>split" lines (returns the count or -errno);
 * unet_tuning_load merges such a file, overriding equal keys (returns the
 * entries read or -errno).  With env UNET_TUNE_DB=<path> the first tuner lookup
 * loads <path> and each newly tuned shape is appended to it. */
int unet_tuning_save(const char* path);
int unet_tuning_load(const char* path);

/* ------------------------------------------------------------------------
 * Per-op entry points (used by the op-level parity tests and by tools).
 * Shapes: x (N,H,W,Ci) NHWC; W OIHW as in PyTorch; outputs NHWC.
 * ---------------------------------------------------------------------- */
/* y = conv3x3_valid(x) + b; optional BN+ReLU transform of x on load
 * (x_scale/x_shift per Ci channel, NULL = identity).  ws >= unet_conv_ws_bytes(). */
int unet_conv3x3_fwd(const float* x, int n, int h, int w, int ci, const float* wt_oihw,
                     const float* bias, int co, const float* x_scale, const float* x_shift,
                     float* y, void* ws, unet_stream_t stream);
/* dx = full-correlation(dy, W) (input gradient).  dy (N,H-2,W-2,Co). */
int unet_conv3x3_dgrad(const float* dy, int n, int h, int w, int ci, const float* wt_oihw,
                       int co, float* dx, void* ws, unet_stream_t stream);
/* dW (OIHW) = sum over pixels of x (x) dy;  db = sum dy. */
int unet_conv3x3_wgrad(const float* x, const float* dy, int n, int h, int w, int ci, int co,
                       float* dw_oihw, float* db, void* ws, unet_stream_t stream);
size_t unet_conv_ws_bytes(int n, int h, int w, int ci, int co);
/* ConvTranspose2d(k=2, s=2): y (N,2H,2W,Co) = convT(x) + b;  W (Ci,Co,2,2). */
int unet_convT2_fwd(const float* x, int n, int h, int w, int ci, const float* wt, const float* bias,
                    int co, float* y, void* ws, unet_stream_t stream);
/* ConvTranspose2d backward: dx, dW (IOHW), db.  ws >= unet_conv_ws_bytes(n,h,w,ci,co). */
int unet_convT2_bwd(const float* x, const float* dy, int n, int h, int w, int ci, const float* wt,
                    int co, float* dx, float* dw, float* db, void* ws, unet_stream_t stream);
/* MaxPool2d(2) floor mode, first max wins; argmax index 0..3 per output. */
int unet_maxpool2_fwd(const float* x, int n, int h, int w, int c, float* y, uint8_t* arg,
                      unet_stream_t stream);
int unet_maxpool2_bwd(const float* dy, const uint8_t* arg, int n, int h, int w, int c, float* dx,
                      unet_stream_t stream);
/* BatchNorm2d train forward over (N,H,W) per channel (+ running-stat update)
 * and backward; y = (x-mean)*invstd*gamma + beta. */
int unet_bn_train_fwd(const float* x, int n, int h, int w, int c, const float* gamma,
                      const float* beta, float* running_mean, float* running_var, float* y,
                      float* save_mean, float* save_invstd, void* ws, unet_stream_t stream);
int unet_bn_train_bwd(const float* x, const float* dy, int n, int h, int w, int c,
                      const float* gamma, const float* save_mean, const float* save_invstd,
                      float* dx, float* dgamma, float* dbeta, void* ws, unet_stream_t stream);
size_t unet_bn_ws_bytes(int c);

/* Building blocks of the reference submodules' own forwards (DoubleConv / Down
 * / Up / OutConv.forward, models/unet_model.py:20-21, 32-33, 50-54, 62-63) and
 * of the op-by-op network path the drop-in takes for a backward through an
 * eval-mode forward.  NHWC tensors unless marked NCHW. */
/* nn.BatchNorm2d (+ the following nn.ReLU when relu != 0): training = batch
 * statistics over (N,H,W), running_mean / running_var updated with `momentum`
 * (unbiased variance), *nbt += 1 (nbt may be NULL); eval = the running
 * statistics.  save_mean / save_invstd receive the statistics used.  c a
 * multiple of 4 dividing 1024. */
size_t unet_bn_relu_ws_bytes(int n, int h, int w, int c);
int unet_bn_relu_fwd(const float* x, int n, int h, int w, int c, const float* gamma, const float* beta,
                     float* running_mean, float* running_var, int64_t* nbt, float momentum, float eps,
                     int training, int relu, float* y, float* save_mean, float* save_invstd, void* ws,
                     unet_stream_t stream);
/* Its backward: y = the forward's output (the ReLU mask), dx, dgamma, dbeta;
 * eval mode treats the statistics as constants (dx = gamma * invstd * dz). */
int unet_bn_relu_bwd(const float* x, const float* y, const float* dy, int n, int h, int w, int c,
                     const float* gamma, const float* save_mean, const float* save_invstd, int training,
                     int relu, float* dx, float* dgamma, float* dbeta, void* ws, unet_stream_t stream);
/* The first conv (any Ci -> 64, 3x3 valid, + bias) from an NCHW input; y NHWC.
 * Backward: dW (OIHW), db, and dx (NCHW; NULL = not needed). */
size_t unet_conv_first_ws_bytes(int n, int ci, int h, int w);
int unet_conv_first_fwd(const float* x_nchw, int n, int ci, int h, int w, const float* wt, const float* bias,
                        float* y, unet_stream_t stream);
int unet_conv_first_bwd(const float* x_nchw, const float* dy, int n, int ci, int h, int w, const float* wt,
                        float* dx_nchw, float* dw, float* db, void* ws, unet_stream_t stream);
/* OutConv's 1x1 conv (64 -> k channels, + bias): logits NCHW; backward dx
 * (NHWC, NULL = not needed), dW (k, 64), db. */
size_t unet_conv1x1_ws_bytes(int k);
int unet_conv1x1_fwd(const float* x, int n, int h, int w, int c, const float* wt, const float* bias, int k,
                     float* logits_nchw, unet_stream_t stream);
int unet_conv1x1_bwd(const float* x, const float* dlogits_nchw, int n, int h, int w, int c, const float* wt, int k,
                     float* dx, float* dw, float* db, void* ws, unet_stream_t stream);

/* Ceilings of this device, measured (bench.py's untimed tail; BASELINE.md asks
 * for roofline fractions against peaks measured on the box): kind 0 = dense
 * bf16 MFMA (v_mfma_f32_32x32x16_bf16) TFLOP/s, 1 = f32 MFMA
 * (v_mfma_f32_16x16x4_f32) TFLOP/s, 2 = HBM float4 copy GB/s (read + write),
 * 3 = HBM read-only stream GB/s.
 * Best of `reps` timed launches after a warm-up; allocates its own buffers. */
int unet_peak_probe(int kind, int reps, double* result, unet_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* UNET_HIP_H */
