// Internal declarations shared by the kernel file and the network plan.
// Not part of the C-ABI (include/unet_hip.h is).
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>
#include <atomic>

namespace unet {

// plan-creation bounds on UNet(n_channels, n_classes) (include/unet_hip.h)
constexpr int kMaxInChannels = 4096;
constexpr int kMaxClassCount = 4096;

// A tensor in NHWC, addressed as an (H, W, C) grid per image with an (oy, ox)
// origin: element (n, y, x, c) lives at ((n*H + y+oy)*W + x+ox)*C + c.
// An optional per-channel affine+ReLU (BatchNorm2d train/eval + nn.ReLU,
// models/unet_model.py:12-17) is applied when the tensor is READ: the network
// stores raw conv outputs and normalises them on load in the consumer.
struct Src {
  const float* ptr = nullptr;
  int H = 0, W = 0, C = 0;   // grid of the stored tensor
  int oy = 0, ox = 0;        // origin added to the pixel position (crop / pad)
  const float* scale = nullptr;  // nullptr: identity
  const float* shift = nullptr;
  // 1: the elements are bf16 (ptr reinterpreted as uint16_t*).  Only tensors
  // that are GEMM operands and nothing else (pooled maps, padded dY, convT
  // output and its gradient) are stored this way, in UNET_PREC_BF16 plans --
  // the GEMMs round them to bf16 anyway -- and never with a transform.
  int h16 = 0;
};

// Implicit-GEMM gather of operand rows: row m enumerates pixels of an
// (Nimg, Hg, Wg) grid; column k enumerates (tap, channel) with
// tap = (ty, tx) in a taps_h x taps_w window and channel in [0, Cg).
// Channels < c_split come from s[0], the rest from s[1] (channel - c_split):
// that is torch.cat([skip_cropped, up], dim=1) (models/unet_model.py:131)
// without a copy.  Source pixel = (y*stride + ty, x*stride + tx) + origin.
struct Gather {
  Src s[2];
  int c_split = 0;      // == Cg when single source
  int Cg = 0;           // channels per tap
  int taps_h = 1, taps_w = 1;
  int stride = 1;
  int Hg = 0, Wg = 0;   // pixel grid of the rows
  int nimg = 0;
};

// Destination of GEMM outputs (fwd/dgrad epilogue), NHWC grid with origin.
struct Dst {
  float* ptr = nullptr;
  int H = 0, W = 0, C = 0;
  int oy = 0, ox = 0;
  int h16 = 0;  // 1: store bf16 (RNE; ptr reinterpreted as uint16_t*)
};

struct Epilogue {
  const float* bias = nullptr;   // per output column
  int shuffle_co = 0;            // >0: ConvTranspose2d k2s2 pixel shuffle
  Dst d[2];
  int n_split = 1 << 30;         // columns < n_split -> d[0], else d[1]
  // eval with BatchNorm folded into the weights (scripts/predict.py's
  // model.eval()): the stored value is relu(conv + folded bias), no statistics
  int relu = 0;
  // forward BN statistics of the stored values: stats[g][col][2] (sum, sumsq)
  double* stats = nullptr;
  // backward: mask the d[0] values with ReLU'(yref*scale+shift) and collect
  // bstats[g][col][2] = (sum dz', sum dz' * xhat), xhat = (yref-mean)*invstd
  const float* yref = nullptr;
  int yref_h16 = 0;  // yref stored bf16 (raw conv outputs of a bf16 plan)
  const float* bn_scale = nullptr;
  const float* bn_shift = nullptr;
  const float* bn_mean = nullptr;
  const float* bn_invstd = nullptr;
  double* bstats = nullptr;
  double* colsum1 = nullptr;     // [g][col - n_split] sums of d[1] values
};

constexpr int kStatGroups = 64;  // fp64 atomic accumulators are spread over groups

struct IgemmArgs {
  Gather a;          // A rows (M = nimg*Hg*Wg pixels), K = taps*Cg
  const float* b = nullptr;      // packed B[N][K] (k contiguous), fp32 tiles
  const uint16_t* bh = nullptr;  // the same packed B in bf16, bf16 tiles (A is
                                 // rounded to bf16 when staged)
  const uint16_t* bl = nullptr;  // split operands (UNET_PREC_BF16X3): B's residual
                                 // plane bf16(B - bh); A is staged as hi/lo too
  int M, N, K;
  Epilogue e;
  // split-K: > 1 slices the K chunks over blockIdx.z; raw partial tiles go to
  // slab[z][M][N] and k_splitk_epi sums them and runs the epilogue
  int ksplit = 1;
  float* slab = nullptr;
  // Winograd F(2x2, 3x3) path (tile 70, winograd.hip): scratch for U, M, V and
  // the variant of its 16 per-point GEMMs
  float* wino_ws = nullptr;
  size_t wino_ws_bytes = 0;
  // batched dense GEMMs (register-staged k_igemm tiles only, no split-K):
  // blockIdx.z = b runs rows b*batch_rows .. (b+1)*batch_rows of the gather
  // (a 1 x (batch*batch_rows) grid), B offset by b*batch_b elements
  int batch = 1;
  int batch_rows = 0;
  long long batch_b = 0;
  struct { int tile = -1, split = 1; } wino_choice;
  // a 3x3 forward conv of the plan (training or eval): held to the forward
  // Winograd caps (g_wino_max, the F(4x4) channel window); every other GEMM
  // (input gradients, convT, op-level calls) to the input-gradient caps
  int fwd = 0;
};

// slab-mode weight gradients that ran with atomics instead (the plan's wslab
// too small for their split partials); unet_slab_fallbacks() reads it
extern std::atomic<long long> g_slab_fallbacks;
// deterministic mode (unet_set_tuning("deterministic", 1), plan.hip): no fp32
// atomics in any weight gradient; sites that had no such variant are counted
extern int g_deterministic;
extern int g_bnb_fuse;
extern int g_wgrad_early_u;  // plan.hip: Winograd weight gradients' U issued before the layer's dY  // plan.hip: fp32 BN-backward apply fused with the F(6x6) dY transform
extern std::atomic<long long> g_nondet_sites;

struct WgradArgs {
  // C[i][j] = sum_p A_p[i] * B_p[j] over the pixels p of the grid of `ga`.
  Gather ga;         // taps = 1: row p -> channels i (contiguous)
  Gather gb;         // row p, column j = (tap, channel)
  int Mo, No;        // output rows (ga.Cg) and cols (gb taps * gb.Cg)
  int P;             // pixels
  int pix_per_split;
  // [Mo][No] fp32.  Atomic modes ADD into it (the caller zeroes it first);
  // slab modes (below) OVERWRITE it: the reduction assigns the sum of the
  // splits, a single split stores straight into it.
  float* out;
  // optional split-partial slab (bf16 ring weight gradients, wgrad per_cu codes
  // >= 10): each pixel split stores its [Mo][No] partial with plain stores and
  // one reduction pass assigns their sum to out -- instead of per_cu x CUs x
  // block fp32 atomics per launch (~9.4 M for every ring launch at 1 per CU)
  float* slab = nullptr;
  size_t slab_bytes = 0;
  // 1: the caller needs out += C (accumulation into earlier contents):
  // launch_wgrad then refuses slab modes (keeps the atomics)
  int accumulate = 0;
  int bf16 = 0;      // 1: operands rounded to bf16 when staged (bf16 tiles 10-14)
  int split = 0;     // 1 (with bf16): operands as hi/lo bf16 pairs (UNET_PREC_BF16X3)
  // batched (fp32 tiles 0-4): blockIdx.z = b * splits + split; operand b's
  // pointers offset by b * batch_a / batch_b elements, its output by b * batch_out
  int batch = 1;
  long long batch_a = 0, batch_b = 0, batch_out = 0;
  // Winograd F(4x4, 3x3) weight gradient (wgrad tile 71, winograd.hip): scratch
  float* wino_ws = nullptr;
  size_t wino_ws_bytes = 0;
  // F(6x6) weight gradient (tile 74) of an fp32 plan: the dY transform Vd was
  // already written here by k_bnb_wino6_dy (fused with the BatchNorm-backward
  // apply); launch_wino_wgrad then skips k_wino6_dy
  const float* vd_pre = nullptr;
  // 1: the Winograd weight gradient's input transform U is already in wino_ws
  // (launch_wino_wgrad_u, issued ahead of the layer's dY)
  int u_ready = 0;
  // timing ablations of k_wgrad3_bf (UNET_WG_ABL; results wrong with any bit):
  // 1 = plain stores instead of the output atomics, 2 = no MFMA, 4 = no operand
  // loads after the first tile
  int abl = 0;
};

// ---------------- launchers (kernels.hip) ----------------
// Variant of a GEMM launch.  igemm: tile id (1-4, 6-9 register-staged,
// 11-14 LDS-DMA staged, 21-26 bf16 operands; see igemm.hip) and K
// split; wgrad: tile id (0-4 fp32, 10-14 bf16) and target workgroups per CU of
// the pixel split.
// tile < 0 = built-in heuristic.  Chosen per launch site by the plan's autotuner.
struct GemmChoice {
  int tile = -1;
  int split = 1;
};
// Winograd F(2x2, 3x3) fp32 path (winograd.hip), tile id 70
size_t wino_ws_bytes(long long T, int Cg, int N);
size_t wino_ws_bytes_grid(int nimg, int H, int W, int Cg, int N);
bool wino_applies(const IgemmArgs& a, int mt);           // mt = 2: F(2x2, 3x3), 4: F(4x4, 3x3)
hipError_t launch_wino(const IgemmArgs& a, hipStream_t s, int mt);
bool wino_wgrad_applies(const WgradArgs& a, int mt);  // weight gradient, mt = 4 (wgrad tile 71) / 6 (74)
bool wino_fused_applies(const IgemmArgs& a);  // tile 72: fused F(4x4, 3x3)
bool wino_fused64_applies(const IgemmArgs& a);  // tile 73: fused F(4x4, 3x3), 64 output channels
hipError_t launch_wino_fused(const IgemmArgs& a, hipStream_t s);
hipError_t launch_wino_fused64(const IgemmArgs& a, hipStream_t s);
bool wino_fused64p_applies(const IgemmArgs& a);  // tile 76: tile 73 on a software-pipelined chunk loop
hipError_t launch_wino_fused64p(const IgemmArgs& a, hipStream_t s);
// tiles 75 / 77: fused F(2x2, 3x3), nc = 64 / 32 output channels x 64 tiles per workgroup
bool wino_fused2_applies(const IgemmArgs& a, int nc);
hipError_t launch_wino_fused2(const IgemmArgs& a, hipStream_t s, int nc);
// MFMA flops a GEMM launch executes with variant c (Winograd: 2 * points *
// tiles * Cg * N; otherwise the direct 2 * M * N * K)
double igemm_exec_flops(const IgemmArgs& a, GemmChoice c);
double wgrad_exec_flops(const WgradArgs& a, GemmChoice c);
hipError_t launch_wino_wgrad(const WgradArgs& a, hipStream_t s, int per_cu, int mt);
int wgrad_winograd_mt(const WgradArgs& a, GemmChoice c);
hipError_t launch_wino_wgrad_u(const WgradArgs& a, hipStream_t s, int mt);  // 4 / 6: the launch is Winograd F(mt x mt); else 0
// fp32 BatchNorm-backward apply fused with the F(6x6) weight gradient's dY
// transform: dYpad (pad 2, border zeroed) and Vd[64][T][c] in one pass
size_t bnb_wino6_vd_bytes(int n, int h, int w, int c);
hipError_t launch_bnb_wino6_dy(const float* dz, const float* y, const float* coef, int n, int h, int w, int c,
                               float* dypad, float* vd, hipStream_t s);
// bf16 halo conv with LDS-DMA weights (conv3_dma.hip), tile ids 63 and 65-68
bool conv3_dma_tile_shape(int tile, int& th, int& bn, int& ch);
hipError_t go_conv3_dma_tile(const IgemmArgs& a, hipStream_t s, int tile);
// bf16 3x3 conv with LDS-DMA halo / weight rings (conv3_ring.hip), tile ids 81-84
// (88: the geometry of 84, persistent)
bool conv3_ring_tile_shape(int tile, int& th, int& bn, int& ck);
bool conv3_ring_fits(const IgemmArgs& a, int tile);
hipError_t go_conv3_ring_tile(const IgemmArgs& a, hipStream_t s, int tile);
hipError_t go_conv3_ring_pt(const IgemmArgs& a, hipStream_t s, int tile);  // conv3_ring_pt.hip (83, 84, 88)
// bf16 convT forward / input gradient on LDS-DMA K rings (gemm_ring.hip), tile ids 91-99
bool gemm_ring_tile_shape(int tile, int& bm, int& bn);
bool gemm_ring_fits(const IgemmArgs& a, int tile);
hipError_t go_gemm_ring_tile(const IgemmArgs& a, hipStream_t s, int tile);
int num_cus();

// Timing-ablation switches (UNET_WG_ABL, UNET_WF_ABL, UNET_WF64_ABL: kernel
// variants with work removed, results WRONG).  They are read only in a build
// with -DUNET_ABLATIONS (make ABLATIONS=1; unet_version() then says
// "ablations"); a production build ignores such a variable and says so once on
// stderr, so a leftover environment can never corrupt a run.
int ablation_env(const char* name);
hipError_t launch_igemm(const IgemmArgs& a, hipStream_t s);  // heuristic
hipError_t launch_igemm_v(const IgemmArgs& a, hipStream_t s, GemmChoice c);
bool igemm_tile_fits(const IgemmArgs& a, int tile);
// workgroups of one K slice and resident workgroups per CU for a tile
long long igemm_tile_count(const IgemmArgs& a, int tile);
int igemm_tile_slots(int tile);
size_t igemm_slab_bytes(const IgemmArgs& a, int ksplit);
hipError_t launch_wgrad(const WgradArgs& a, hipStream_t s);  // heuristic
hipError_t launch_wgrad_v(const WgradArgs& a, hipStream_t s, GemmChoice c);
bool wgrad_tile_fits(const WgradArgs& a, int tile);
// bf16-operand kernels (igemm_bf16.hip), dispatched by the launchers above
hipError_t go_igemm_bf16(const IgemmArgs& a, hipStream_t s, int tile);
// halo-tiled 3x3 tiles 31-36: output tile TH x TW pixels x BN columns
bool halo_tile_shape(int tile, int& th, int& tw, int& bn);
hipError_t go_wgrad_bf16(const WgradArgs& a, hipStream_t s, int tile, dim3 grid);
// halo-tiled 3x3 weight gradient (wgrad tiles 20, 21): all 9 taps per workgroup
bool wgrad3_fits(const WgradArgs& a);
hipError_t go_wgrad3_bf16(const WgradArgs& a, hipStream_t s, int tile, int per_cu);
// 3x3 weight gradient with every operand staged by LDS-DMA through a 4-slot
// ring of pixel tiles (wgrad tiles 26-33, wgrad3_ring.hip)
bool wgrad3_ring_fits(const WgradArgs& a, int tile);
hipError_t go_wgrad3_ring(const WgradArgs& a, hipStream_t s, int tile, int per_cu);
// out[b][e] = sum_z slab[b * splits + z][e], e < plane (the slab-mode weight
// gradients' reduction; out planes batch_out floats apart)
hipError_t launch_slab_reduce(const float* slab, int splits, int batch, size_t plane, long long batch_out, float* out,
                              hipStream_t s);
// pixel splits of a pixel-column weight-gradient tile (and the pixels per split)
int wgrad_splits(const WgradArgs& a, int tile, int per_cu, int& pps);
// whether slab mode can hold `splits` partial planes (1 split: stores into out)
bool wgrad_slab_fits(const WgradArgs& a, int splits);
// wide halo-tiled 3x3 weight gradient with a two-stage ring (wgrad tiles 24, 25)
bool wgrad3w_fits(const WgradArgs& a, int tile);
hipError_t go_wgrad3w_bf16(const WgradArgs& a, hipStream_t s, int tile, int per_cu);
// tiles 21-26 / 31-36 / 41-44 that have a split-operand kernel
bool bf16_tile_splits(int tile);
// out[i] = bf16(in[i]) (RNE), n a multiple of 4, in 16-B / out 8-B aligned;
// lo (optional): lo[i] = bf16(in[i] - out[i]), the residual plane of split operands
hipError_t launch_f2bf(const float* in, uint16_t* out, size_t n, hipStream_t s, uint16_t* lo = nullptr);

// overlap-tile gather / scatter (tiling.hip)
hipError_t launch_tile_gather(const float* img, int c, int h, int w, int ti, int to, int top, int left, int nx,
                              int first, int stride, int ntiles, float* tiles, hipStream_t s);
hipError_t launch_tile_scatter(const float* lt, int k, int to, int nx, int first, int stride, int ntiles, int h,
                               int w, float* full, uint8_t* mask, hipStream_t s);

// post-processing (postproc.hip)
size_t instance_masks_ws_bytes(int n, int h, int w);
hipError_t launch_instance_masks(const uint8_t* mask, int n, int h, int w, int min_size, uint16_t* out, void* ws,
                                 hipStream_t s);
size_t rand_index_ws_bytes(int h, int w);
hipError_t launch_rand_index(const uint16_t* g, const uint16_t* p, int h, int w, double* out, void* ws,
                             hipStream_t s);

// loss weight maps (weightmap.hip)
size_t weight_map_ws_bytes(int n);
hipError_t launch_weight_map(const uint16_t* lab, int n, int h, int w, double w0, double sigma, float* out,
                             double* out64, void* ws, hipStream_t s);

// elastic-deformation input pipeline (elastic.hip)
size_t elastic_ws_bytes(int n, int h, int w);
hipError_t launch_elastic(const uint8_t* img, const uint16_t* lab, int n, int h, int w, const double* noise,
                          double alpha, double sigma, float* x_out, uint8_t* t_out, uint8_t* img_out, void* ws,
                          hipStream_t s);

// inc.c0: Ci in {1,2,3,4} direct conv from an NCHW input; y NHWC (Co = 64 multiple).
hipError_t launch_conv_first_fwd(const float* x_nchw, int n, int ci, int h, int w,
                                 const float* wt_oihw, const float* bias, int co, float* y,
                                 double* stats, hipStream_t s, int out_h16 = 0, int relu = 0);
// eval BatchNorm fold: wout[r][:] = w[r][:] * scale[r], bias_out[r] = scale[r] * bias[r] + shift[r]
hipError_t launch_fold_bn(const float* w, long long K, int rows, const float* scale, const float* shift,
                          const float* bias, float* wout, float* bias_out, hipStream_t s);
// Written per workgroup into `slabs` (conv_first_wgrad_ws_bytes) then reduced
// into dw_oihw (overwritten, not accumulated).
constexpr int kFirstWgradSlabs = 2048;
size_t conv_first_wgrad_ws_bytes(int ci);
hipError_t launch_conv_first_wgrad(const float* x_nchw, int n, int ci, int h, int w,
                                   const Src& dy, int co, float* dw_oihw, float* slabs, hipStream_t s);
// inc.c0 weight gradient with the BN0 backward fused in (reads dz, y, x; coef =
// k_bnb_finalize's [k0|k1|k2|mean] per channel)
hipError_t launch_conv_first_wgrad_bn(const float* x, int n, int ci, int h, int w, const float* dz, const float* y,
                                      int y_h16, const float* coef, int co, float* dw, float* slabs, hipStream_t s,
                                      int dz_h16 = 0);

// BN finalize (train): stats[G][C][2] -> mean, invstd, scale, shift; running update.
hipError_t launch_bn_finalize(const double* stats, int c, double count, const float* gamma,
                              const float* beta, float* rmean, float* rvar, int64_t* nbt,
                              float* mean, float* invstd, float* scale, float* shift,
                              float momentum, float eps, hipStream_t s);
// BN eval prepare: scale/shift from running stats.
hipError_t launch_bn_eval_prepare(int c, const float* gamma, const float* beta,
                                  const float* rmean, const float* rvar, float* scale,
                                  float* shift, float eps, hipStream_t s);
// BN backward finalize: bstats -> dgamma, dbeta, conv-bias grad, coefficients
// k[3][C] for dY = k0*dz' + k1*y + k2.
hipError_t launch_bnb_finalize(const double* bstats, int c, double count, const float* gamma,
                               const float* mean, const float* invstd, float* dgamma,
                               float* dbeta, float* dbias_conv, float* coef, hipStream_t s, int eval = 0);
// dYpad interior = coef0*dz + coef1*y + coef2; border (pad each side) = 0.
hipError_t launch_bnb_apply(const float* dz, const float* y, const float* coef, int n, int h,
                            int w, int c, float* dypad, int pad, hipStream_t s, int out_h16 = 0,
                            int y_h16 = 0, int dz_h16 = 0);
// MaxPool2d(2) fwd with BN+ReLU transform on load (src grid H x W, pooled H/2 x W/2);
// anorm (bf16 plans): also writes every window element's relu(bn(.)) in bf16.
hipError_t launch_maxpool_fwd(const Src& src, int n, int h, int w, float* y, uint8_t* arg,
                              hipStream_t s, int out_h16 = 0, uint16_t* anorm = nullptr);
// a = bf16(relu(y * scale + shift)), y bf16 NHWC (pixels x c, c % 8 == 0)
hipError_t launch_bn_relu_bf(const uint16_t* y, const float* scale, const float* shift, long long pixels, int c,
                             uint16_t* a, hipStream_t s);
// Maxpool bwd fused: dz = route(dpool) + crop-embedded dskip (may be null), then
// ReLU mask + BN-bwd stats (if scale != null).  Writes dz' (n,h,w,c).
hipError_t launch_maxpool_bwd_fused(const float* dpool, const uint8_t* arg, const float* dskip,
                                    int skip_oy, int skip_ox, int skip_h, int skip_w,
                                    const float* y, const float* scale, const float* shift,
                                    const float* mean, const float* invstd, int n, int h, int w,
                                    int c, float* dz, double* bstats, hipStream_t s, int y_h16 = 0,
                                    int g_h16 = 0);
// 1x1 head (OutConv, models/unet_model.py:56-63) forward: logits NCHW.
hipError_t launch_head_fwd(const Src& src, int n, int h, int w, int c, const float* wt,
                           const float* bias, int k, float* logits, hipStream_t s);
// 1x1 conv backward on a plain fp32 NHWC input (64 channels): dx (nullable), dW, db
hipError_t launch_head_bwd_plain(const float* x, const float* dl, int n, int h, int w, const float* wt, int k,
                                 float* dx, float* dw, float* db, double* acc, hipStream_t s);
// inc.c0 input gradient, dx NCHW (per-op path only)
hipError_t launch_conv_first_dgrad(const float* dy, int n, int ci, int h, int w, const float* wt, float* dx,
                                   hipStream_t s);
// head backward: dz' (masked, + BN-bwd stats), dW (k x c), db (k) (written, not accumulated).
hipError_t launch_head_bwd(const Src& src, const float* dlogits, int n, int h, int w, int c,
                           const float* wt, int k, const float* yraw, const float* mean,
                           const float* invstd, float* dz, double* bstats, float* dw, float* db,
                           double* ws_acc, hipStream_t s, int dz_h16 = 0);
hipError_t launch_wce(const float* logits, const int64_t* t, const float* wm, int n, int k, int h,
                      int w, const int64_t* ts, const int64_t* wsd, float* loss, float* dlogits,
                      float grad_scale, double* acc, hipStream_t s);
hipError_t launch_sgd(float* p, const float* g, float* buf, size_t n, float lr, float mom,
                      float gscale, int first, hipStream_t s);
hipError_t launch_scale_by_dev(const float* x, float* y, size_t n, const float* g, hipStream_t s);
// weight repacks
hipError_t launch_pack_conv(const float* w_oihw, int co, int ci, int kh, int kw, float* wf,
                            float* wd, hipStream_t s);
hipError_t launch_pack_convT(const float* w, int ci, int co, float* wf, float* wd, hipStream_t s);
// all of a forward's conv / convT weight repacks in one launch (k_pack_all)
struct PackJob {
  const float* w;  // conv: W[co][ci][9] (OIHW); convT: W[ci][co][4]
  float* wf;       // conv: [co][9][ci]; convT: [4*co][ci]
  float* wd;       // conv: [ci*9 + 8-t][co] (nullptr: eval, not needed); convT: [ci][4][co]
  int co, ci, kind;  // kind 0 conv 3x3, 1 convT 2x2 s2; co, ci multiples of 32
};
constexpr int kPackJobsMax = 24;
struct PackJobs {
  PackJob j[kPackJobsMax];
  int first[kPackJobsMax + 1];
  int n;
};
hipError_t launch_pack_all(PackJobs jobs, hipStream_t s);
// out[a][c][b] = in[a][b][c]
hipError_t launch_permute_last2(const float* in, int A, int B, int C, float* out, hipStream_t s);
// column sums over rows: out[c] = sum_r in[r][c] via double groups
hipError_t launch_colsum(const double* groups, int g, int c, float* out, hipStream_t s);
hipError_t launch_iou(const uint8_t* a, const uint8_t* b, size_t n, unsigned long long* out,
                      hipStream_t s);
hipError_t launch_mask(const float* logits, uint8_t* mask, int n, int h, int w, hipStream_t s);
// generic BN stats over an NHWC tensor (per-op BN API)
hipError_t launch_channel_stats(const float* x, size_t pixels, int c, double* stats,
                                hipStream_t s);
hipError_t launch_affine_relu(const float* x, size_t pixels, int c, const float* scale,
                              const float* shift, int relu, float* y, hipStream_t s);
hipError_t launch_bn_bwd_stats(const float* dy, const float* x, const float* mean,
                               const float* invstd, size_t pixels, int c, double* bstats,
                               hipStream_t s);

}  // namespace unet
