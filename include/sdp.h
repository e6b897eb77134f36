/*
 * sdp.h -- C ABI of libsdp.so, the MI355X (gfx950) implementation of the
 * Simultaneous-Diffusion-for-Pointclouds sampling hot path.
 *
 * Every pointer argument named x/grad/ref/... is a DEVICE pointer owned by the caller
 * unless documented otherwise; every call is enqueued on the caller's hipStream_t
 * (passed as void*) and never synchronises the device.  Return value: 0 = OK,
 * < 0 = error; sdp_last_error() gives a thread-local message for the last failure.
 * Handles are per device and not thread-safe: one handle per (device, thread).
 *
 * Reference interfaces replaced (paths relative to /root/reference/LiDARGen):
 *   sdp_net_*              scorenet(x, y) = NCSN_LiDAR_small.forward   models/ncsnv2.py:420-518
 *                          weight load    load_state_dict + EMAHelper  runners/ncsn_runner_kitti_simultaneous.py:472-489
 *   sdp_langevin_step      Langevin update                           models/KITTISampling.py:133-156,
 *   sdp_net_forward_langevin  scorenet + Langevin update in one call   models/KITTISampling.py:137-156
 *                                                                     models/__init__.py:236-259, :1397-1416
 *   sdp_consistency_merge  cross-view reprojection + correction      models/KITTISampling.py:160-490 (pose matrices),
 *                                                                     models/__init__.py:263-579 (origin offsets)
 *   sdp_net_forward_train  scores = scorenet(perturbed, labels) in train mode   losses/dsm.py:85
 *   sdp_dsm_loss           anneal_dsm_score_estimation_with_mask            losses/dsm.py:67-119
 *   sdp_net_backward       loss.backward()                                  runners/ncsn_runner_kitti_simultaneous.py:230
 *   sdp_net_backward_buckets  loss.backward() + DataParallel's gradient reduce  (kitti runner :104,481,230)
 *   sdp_adam_ema_step      optimizer.step() (Adam, losses/__init__.py:10-20) + EMAHelper.update (models/ema.py:16-21)
 *   sdp_optim_ema_step     optimizer.step() of Adam / RMSprop / SGD (get_optimizer, losses/__init__.py:3-13) + EMA
 *   sdp_range_project      point_cloud_to_range_image                       datasets/lidar_utils.py:54-347
 *   sdp_view_transform     pose chain fromWorld @ (toWorld @ p)             datasets/kitti360_im_8Batch.py:146-190
 *   sdp_view_gather        scanPoints[index[index >= 0]]                    datasets/kitti360_im_simultenous_densification.py:186-203
 *   sdp_view_finalize      __getitem__ post-processing of the range images  datasets/kitti360_im_8Batch.py:221-304
 *   sdp_grid_subsample     voxel-grid subsampling (HOST)                    datasets/cpp_wrappers/cpp_subsampling/
 *                                                                             grid_subsampling{,_lidar}.cpp, wrapper.cpp:58-285
 */
#ifndef SDP_H
#define SDP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SDP_VERSION 100  /* 1.0.0 */

/* arithmetic used for the score network's convolutions (fp32 I/O and accumulation in all modes) */
enum sdp_precision {
  SDP_PREC_FP32 = 0,    /* v_mfma_f32_32x32x2_f32: exact fp32 products                         */
  SDP_PREC_FP32X3 = 1,  /* 3-pass bf16 split (hi*hi + hi*lo + lo*hi) on v_mfma_f32_16x16x32_bf16  */
                        /* (forward and data gradient; weight gradient on v_mfma_f32_32x32x16)   */
  SDP_PREC_BF16 = 2     /* single bf16 pass (fast, NOT within the fp32 parity tolerance)        */
};

typedef struct sdp_net_desc {
  int ngf;          /* 128 (NCSN_LiDAR_small config.model.ngf)                    */
  int channels;     /* 2 (depth, intensity)                                        */
  int H, W;         /* 64, 1024 (config.data.image_size / image_width)             */
  int num_classes;  /* 232 (length of the model's sigma buffer)                    */
  int precision;    /* enum sdp_precision                                          */
} sdp_net_desc;

typedef struct sdp_net sdp_net;

int sdp_version(void);
const char* sdp_last_error(void);

/* ---- score network (NCSN_LiDAR_small) ------------------------------------------------ */
int sdp_net_create(const sdp_net_desc* desc, sdp_net** out);
/* Copy one state_dict tensor (HOST float32, reference key and shape, e.g. "res1.0.conv1.weight"
 * [128,128,3,3] or "sigmas" [232]).  The library owns its copy after the call. */
int sdp_net_set_param(sdp_net* net, const char* key, const float* host_data, const int64_t* shape, int ndim);
/* Check every parameter was set and upload the device layouts (blocking; call once). */
int sdp_net_finalize(sdp_net* net);
int sdp_net_workspace_size(const sdp_net* net, int B, size_t* bytes);
/* out[B,2,H,W] = scorenet(x[B,2,H,W], labels[B]) ; labels: int64 device array indexing sigmas. */
int sdp_net_forward(sdp_net* net, const float* x, const int64_t* labels, float* out, int B,
                    void* workspace, size_t workspace_bytes, void* stream);
int sdp_net_destroy(sdp_net* net);
/* One annealed-Langevin step with the update fused into the score net's last kernel
 * (KITTISampling.py:137-156 in one call): grad = scorenet(x, labels) is computed and, in the same
 * epilogue, x <- x + step*g' + grad_ref*lik + noise*noise_scale exactly as sdp_langevin_step
 * (same float32 order, same Philox counters: bit-identical to sdp_net_forward followed by
 * sdp_langevin_step).  x [B,2,H,W] is read by the first layer and updated in place by the last.
 * grad_out (nullable) receives the scores; lik_out / absmax_bits as in sdp_langevin_step.     */
typedef struct {
  const float* ref;            /* [B,2,H,W] */
  const int32_t* mask;         /* [B,2,H,W] */
  const float* noise;          /* nullable: Philox4x32-10(seed, offset + i/4) */
  uint64_t seed, offset;
  float step_size, noise_scale, grad_ref;
  int nan_to_num;
  float* lik_out;              /* nullable */
  uint32_t* absmax_bits;       /* nullable */
  float* grad_out;             /* nullable */
} sdp_langevin_params;
int sdp_net_forward_langevin(sdp_net* net, float* x, const int64_t* labels, int B, const sdp_langevin_params* params,
                             void* workspace, size_t workspace_bytes, void* stream);
/* Performance knob: run sdp_net_forward / sdp_net_forward_langevin as `ways` part-batch forwards on
 * that many streams (the caller's + the handle's own, joined before return; 1 = one launch per
 * layer, 0 = the default, 2).  Results are identical for every value; the
 * workspace size depends on it (query sdp_net_workspace_size after setting it).              */
int sdp_net_set_split(sdp_net* net, int ways);
/* Measurement hooks: when enabled, every conv launch of sdp_net_forward is bracketed by HIP
 * events on the forward's stream; sdp_net_profile_read synchronises on them and writes one
 * line per conv class: "class\tlaunches\ttotal_ms\tflops_per_launch\n". */
int sdp_net_profile_enable(sdp_net* net, int enable);
int sdp_net_profile_read(sdp_net* net, char* buf, size_t cap, int* n_launches);

/* ---- parameters as one device arena (training) ------------------------------------------
 * Every learnable parameter (state_dict keys minus the "sigmas" buffer), float32, each at a
 * 64-float aligned offset, in the order sdp_net_backward finishes their gradients (head first,
 * begin_conv last; sdp_net_param_info enumerates it).  sdp_net_bind_params copies the current values into a
 * caller-owned device arena of sdp_net_param_arena_floats floats and makes it the net's
 * parameter storage; after the caller changes it (optimizer), sdp_net_repack rebuilds the
 * packed conv weights on `stream`.  Gradient arenas use the same layout.                    */
int sdp_net_param_arena_floats(const sdp_net* net, size_t* n);
int sdp_net_param_count(const sdp_net* net, int* n);
int sdp_net_param_info(const sdp_net* net, int i, char* key, size_t cap, size_t* offset, size_t* numel);
int sdp_net_bind_params(sdp_net* net, float* arena, void* stream);
int sdp_net_repack(sdp_net* net, void* stream);

/* ---- DSM training (BASELINE config 5; precision fp32x3 or bf16) -------------------------
 * sdp_net_forward_train: out = scorenet(x, labels), keeping every tensor the backward needs
 * (the tape) in `workspace` (sdp_net_train_workspace_size bytes).  sdp_net_backward then writes
 * d loss/d parameters for d loss/d out = dscore into `grads` (a parameter-layout arena,
 * overwritten) -- same workspace and B, no other train-mode call on this net in between.   */
int sdp_net_train_workspace_size(sdp_net* net, int B, size_t* bytes);
/* bf16 precision only: 1 (the default) keeps the tape -- every activation and output gradient of
 * sdp_net_forward_train / sdp_net_backward -- in bf16 (half the bytes of every conv's operand and
 * epilogue streams, of the weight gradient's and of the adjoints'); 0 keeps it in float32.  The
 * parameters, the gradient arena, the statistics and the scores are float32 either way.  Takes effect
 * at the next sdp_net_train_workspace_size / sdp_net_forward_train (the workspace size depends on it). */
int sdp_net_set_tape(sdp_net* net, int bf16);
int sdp_net_forward_train(sdp_net* net, const float* x, const int64_t* labels, float* out, int B,
                          void* workspace, size_t workspace_bytes, void* stream);
int sdp_net_backward(sdp_net* net, const float* dscore, int B, void* workspace, size_t workspace_bytes,
                     float* grads, void* stream);
/* sdp_net_backward with gradient buckets for a data-parallel reduce overlapped with the backward
 * (replaces the implicit gradient reduce of torch.nn.DataParallel,
 * runners/ncsn_runner_kitti_simultaneous.py:104,481): bucket i is the arena range
 * [bucket_end[i-1], bucket_end[i]) (floats, increasing, <= sdp_net_param_arena_floats); events[i]
 * (hipEvent_t) is recorded on `stream` as soon as the launches that finish every gradient of that
 * range are enqueued, so a communication stream can wait on it while the backward goes on. */
int sdp_net_backward_buckets(sdp_net* net, const float* dscore, int B, void* workspace, size_t workspace_bytes,
                             float* grads, int n_buckets, const size_t* bucket_end, void* const* events,
                             void* stream);
/* loss = mean_b 1/2 * sum_i (mask*(score - target))^2 * n_img / sum(mask) * sigma_b^p with
 * target = -noise / sigma_b^2 (noise already scaled by sigma_b, as the reference passes it);
 * writes dscore = d loss / d score, loss[0], loss_per[b] (optional).  mask float32 0/1,
 * n_img = C*H*W, part: 2*B*64 floats of scratch.                                             */
int sdp_dsm_loss(const float* score, const float* noise, const float* mask, const float* used_sigma, int B,
                 int n_img, float anneal_power, float* dscore, float* loss, float* loss_per, float* part,
                 void* stream);
/* torch.optim.Adam step (weight_decay 0, amsgrad off) over n floats, step = 1, 2, ...; then
 * ema_shadow = (1 - ema_mu)*p + ema_mu*ema_shadow if ema_shadow is not NULL.                 */
int sdp_adam_ema_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, float* ema_shadow,
                      size_t n, double lr, double beta1, double beta2, double eps, int step, double ema_mu,
                      void* stream);
/* optimizer.step() of every optimizer get_optimizer builds (losses/__init__.py:3-13), in torch's
 * per-element order, then the EMA update as above.  g <- g + weight_decay*p first (all kinds).
 *   SDP_OPTIM_ADAM    state0 exp_avg, state1 exp_avg_sq, state2 max_exp_avg_sq (amsgrad) or NULL;
 *                     betas (beta1, beta2)
 *   SDP_OPTIM_RMSPROP state0 square_avg; beta2 = alpha (torch default 0.99), eps (default 1e-8)
 *   SDP_OPTIM_SGD     state0 momentum_buffer (written as g on step 1); beta1 = momentum, dampening 0
 * step = 1, 2, ... (the optimizer's step count after this step).                            */
enum sdp_optim_kind { SDP_OPTIM_ADAM = 0, SDP_OPTIM_RMSPROP = 1, SDP_OPTIM_SGD = 2 };
int sdp_optim_ema_step(int kind, float* params, const float* grads, float* state0, float* state1, float* state2,
                       float* ema_shadow, size_t n, double lr, double beta1, double beta2, double eps,
                       double weight_decay, int step, double ema_mu, void* stream);
/* (hyperparameters are host doubles -- the Python floats torch.optim and EMAHelper compute with:
 *  1 - beta, 1 - mu and the bias corrections are formed in double and rounded once)          */

/* ---- Langevin update ------------------------------------------------------------------ *
 * x <- x + step*g' + grad_ref*lik + noise*noise_scale   (float32, reference evaluation order)
 *   g'  = nan_to_num(grad) if nan_to_num else grad;  lik = -mask*(x - ref)
 *   noise = noise_or_null[i] if given, else N(0,1) from Philox4x32-10(seed, counter = offset + i/4)
 * Optional outputs: lik_out (the step's grad_likelihood, used by the denoise step) and
 * absmax_bits: atomicMax of |x_new[:,0]| float bits (the merge's tooHigh input).          */
int sdp_langevin_step(float* x, const float* grad, const float* ref, const int32_t* mask,
                      const float* noise_or_null, uint64_t seed, uint64_t offset,
                      float step_size, float noise_scale, float grad_ref, int nan_to_num,
                      int B, int C, int HW, float* lik_out, uint32_t* absmax_bits, void* stream);
/* x <- x + a*g + b*lik   (denoise: a = sigma_L^2, b = grad_ref) ; x <- x + b*(-mask*(x-ref)) if g == NULL */
int sdp_axpy_step(float* x, const float* g, float a, const float* lik, const int32_t* mask,
                  const float* ref, float b, int n, void* stream);

/* ---- cross-view consistency merge ----------------------------------------------------- */
enum sdp_merge_variant { SDP_MERGE_POSES = 0, SDP_MERGE_ORIGINS = 1 };

typedef struct sdp_merge_params {
  int variant;            /* enum sdp_merge_variant                                        */
  int setting;            /* 5 (kitti min-depth filter) / 7 (AllForOne controlled average) */
  float sigma;            /* current sigma (float32 from the sigma array)                  */
  float allowance;        /* metres (10)                                                   */
  float cc;               /* correlation coefficient                                       */
} sdp_merge_params;

int sdp_merge_workspace_size(int n_src, int n_out, int H, int W, size_t* bytes);   /* any aB <= n_src */
/* the same for megabatches of exactly aB views (the pair records scale with n_out * aB * H * W) */
int sdp_merge_workspace_bytes(int n_src, int aB, int n_out, int H, int W, size_t* bytes);
/*
 * x_all   : [n_src,2,H,W] current images of every source view (device, float32)
 * toWorld : [n_src,4,4] float64 (POSES) ; fromWorld : [n_src,4,4] float64 (POSES)
 * origins : [aB,3] float32 view origins (ORIGINS variant; models/__init__.py:224-231)
 * exist   : [aB,H,W] uint8 (existMask[:aB]) ; sky : [n_src,H,W] uint8 ; refmask : [n_src,2,H,W] int32
 * Views are grouped into megabatches of aB consecutive indices.  Output views are
 * [o_begin, o_begin+n_out); their images in x_all are corrected in place.
 * absmax_bits : device word holding max|x[:,0]| bits over ALL views of the step (tooHigh).
 * new_images  : optional [n_out,2,H,W] float32 output (the reference's newImages).
 */
int sdp_consistency_merge(float* x_all, int n_src, int aB, int o_begin, int n_out, int H, int W,
                          const double* toWorld, const double* fromWorld, const float* origins,
                          const uint8_t* exist, const uint8_t* sky, const int32_t* refmask,
                          const sdp_merge_params* params, const uint32_t* absmax_bits,
                          float* new_images, void* workspace, size_t workspace_bytes, void* stream);
/* The same merge for multi-rank runs: the stream waits for absmax_event (a hipEvent_t
 * recorded after the cross-rank all_reduce(MAX) of absmax_bits, or NULL) only right before the final
 * correction pass, the merge's one reader of that word -- so the all_reduce on another stream runs
 * beside the projection, binning and resolve passes instead of before them. */
int sdp_consistency_merge_ev(float* x_all, int n_src, int aB, int o_begin, int n_out, int H, int W,
                             const double* toWorld, const double* fromWorld, const float* origins,
                             const uint8_t* exist, const uint8_t* sky, const int32_t* refmask,
                             const sdp_merge_params* params, const uint32_t* absmax_bits,
                             float* new_images, void* workspace, size_t workspace_bytes, void* stream,
                             void* absmax_event);

/* ---- point cloud -> range image (data front end; datasets/lidar_utils.py:54-347) --------
 * points: DEVICE float64 [N][stride] (x, y, z[, intensity]); origin: HOST float64 [3].
 * Outputs (DEVICE, [H][W], already flipped in both axes like the reference): depth float64
 * (maxRange 2057.701 where empty), intensity float64 (optional, needs has_intensity),
 * obfuscation u8, sky u8 (all 0, as the reference clears it; both NULL skips the row-sequential
 * sky/obfuscation scan), index int64 (optional, -1 empty).
 * The nearest point per pixel wins; equal depths keep the lowest point index.               */
int sdp_range_project_workspace_size(int H, int W, size_t* bytes);
int sdp_range_project(const double* points, int N, int stride, int has_intensity, const double* origin,
                      int H, int W, double* depth, double* intensity, uint8_t* obfuscation, uint8_t* sky,
                      int64_t* index, void* workspace, size_t workspace_bytes, void* stream);

/* ---- KITTI-360 view rendering (the datasets' __getitem__) --------------
 * sdp_view_transform: points DEVICE float32 [n][4] (x, y, z, intensity, the .bin layout);
 *   m1, m2 HOST float64 row-major 4x4 or NULL.  out DEVICE float64 [n][4] =
 *   (m2 @ (m1 @ [x y z 1]))[:3], intensity -- kitti360_im_8Batch.py:146-190 with m1 = toWorld
 *   of the scan's pose and m2 = fromWorld of the goal pose; NULL, NULL = float64 widening.
 * sdp_view_gather: the densification subsample scanPoints[index[index >= 0]] after
 *   index[:, :blank_cols] = -2 (kitti360_im_simultenous_densification.py:186-203).  index DEVICE
 *   int64 [H][W] (sdp_range_project output), points DEVICE float32 [N][4]; out DEVICE float64
 *   [<= H*W][4] in row-major pixel order; *count (DEVICE int) = number written.
 * sdp_view_finalize: kitti360_im_8Batch.py:221-304 (variant SDP_VIEW_8BATCH),
 *   kitti360_im_AllForOne.py:253-353 (SDP_VIEW_ALLFORONE), kitti360_im_simultenous_
 *   densification.py:230-339 (SDP_VIEW_DENSIFICATION; first_view = numberInBatch == 0).
 *   Inputs are sdp_range_project outputs of the view and of the goal scan ([H][W], DEVICE;
 *   intensity / goal_intensity only with channels == 2); roll = the random_roll column shift
 *   or -1.  Outputs DEVICE: real, goal float64 [channels][H][W], notmask u8 [channels][H][W]
 *   (np.logical_not(mask)), notsky u8 [H][W] (np.logical_not(sky) after the 3-row shift).
 *   SDP_VIEW_COMPLETION: kitti360_im_SceneCompletion.py:388-513 -- channel 2 of real is the
 *   depth code again and its mask is all ones (the reference concatenates (real, real) and
 *   (mask, ones)); goal_depth / goal_intensity / goal may be NULL (no goal scan).            */
enum sdp_view_variant { SDP_VIEW_8BATCH = 0, SDP_VIEW_ALLFORONE = 1, SDP_VIEW_DENSIFICATION = 2, SDP_VIEW_COMPLETION = 3 };
int sdp_view_transform(const float* points, int64_t n, const double* m1, const double* m2, double* out, void* stream);
int sdp_view_gather(const int64_t* index, int H, int W, int blank_cols, const float* points, double* out, int* count,
                    void* stream);
int sdp_view_finalize(const double* depth, const double* intensity, const uint8_t* obfuscation, const uint8_t* sky,
                      const double* goal_depth, const double* goal_intensity, int H, int W, int channels, int roll,
                      int variant, int first_view, double* real, uint8_t* notmask, uint8_t* notsky, double* goal,
                      void* stream);

/* ---- §8(f)-3: voxel-grid subsampling, HOST memory (no stream) ------------------------------
 * sdp_grid_subsample replaces the CPython modules grid_subsampling.compute (method 0,
 *   "barycenters": grid_subsampling.cpp:46-102) and grid_subsampling_lidar.compute (method 1:
 *   grid_subsampling_lidar.cpp:46-120), wrapper.cpp:58-285.  points float32 [n][3], features
 *   float32 [n][fdim] or NULL, classes int32 [n][ldim] or NULL, voxel size sample_dl.  Outputs
 *   (capacity n rows each): out_points [m][3], out_features [m][fdim], out_classes [m][ldim];
 *   *out_n = m, in the reference's voxel order (see csrc/grid_subsampling.cpp).             */
int sdp_grid_subsample(const float* points, int64_t n, const float* features, int fdim, const int32_t* classes,
                       int ldim, float sample_dl, int method, float* out_points, float* out_features,
                       int32_t* out_classes, int64_t* out_n);

#ifdef __cplusplus
}
#endif
#endif
