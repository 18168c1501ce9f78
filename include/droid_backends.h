/*
 * droid_backends.h — C ABI of the MI355X-native replacement for the
 * reference's `droid_backends` CUDA extension (src/droid.cpp:237-250).
 *
 * Library: droid-slam_amd/lib/libdroid_hip.so (hipcc --offload-arch=gfx950).
 * All pointers are DEVICE pointers unless marked "host"; every tensor is
 * dense row-major (C-contiguous) in the layout the reference uses.  Calls are
 * asynchronous on `stream` (a hipStream_t; pass the caller's current stream).
 * Every function returns 0 on success, non-zero on error; the message is in
 * droid_last_error() (thread local).  No torch types cross this boundary.
 */
#ifndef DROID_BACKENDS_H
#define DROID_BACKENDS_H

#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes */
#define DROID_OK 0
#define DROID_INVALID_ARGUMENT 1
#define DROID_UNSUPPORTED 2
#define DROID_HIP_ERROR 3

/* dtype codes for the correlation entry points */
#define DROID_F16 0
#define DROID_F32 1
#define DROID_F64 2

const char* droid_last_error(void);
int droid_abi_version(void);
int droid_device_count(void);
/* bit 0: the A/B build (`make ab`: dropped kernel variants + DROID_* experiment
 * knobs), bit 1: the profiling build (`make prof`); 0 for the product library,
 * which takes no kernel choice from the environment */
int droid_build_info(void);

/* ---- correlation -------------------------------------------------------- */

/* replaces corr_index_forward  (src/droid.cpp:170-178, correlation_kernels.cu:126-155)
 * volume (B,H,W,H2,W2) dtype, coords (B,2,H,W) f32 -> corr (B,2r+1,2r+1,H,W) dtype.
 * corr[:,i,j] = bilinear sample at (x0-r+i, y0-r+j), zero outside; fp16 is
 * bit-exact with the reference's at::Half arithmetic. */
int droid_corr_index_forward(int dtype, const void* volume, const float* coords, void* corr,
                             int B, int H, int W, int H2, int W2, int radius, hipStream_t stream);

/* replaces corr_index_backward (src/droid.cpp:180-191, correlation_kernels.cu:157-185)
 * volume_grad must be zero-initialised (B,H,W,H2,W2). */
int droid_corr_index_backward(int dtype, const float* coords, const void* corr_grad,
                              void* volume_grad, int B, int H, int W, int H2, int W2, int radius,
                              hipStream_t stream);

/* CorrBlock.__call__ (modules/corr.py:40-50) for all pyramid levels in one launch:
 * levels[l] (E,H,W,H2s[l],W2s[l]), coords (E,H,W,2) f32 at level-0 scale
 * -> out (E, num_levels*(2r+1)^2, H, W), identical to cat of per-level lookups. */
int droid_corr_pyramid_lookup(int dtype, const void* const* levels, const int* H2s, const int* W2s,
                              int num_levels, const float* coords, void* out, int E, int H, int W,
                              int radius, hipStream_t stream);

/* CorrBlock.__call__ (modules/corr.py:40-50; fp16, r=3) over the 8x8-tiled slot
 * pool of CorrBlock(tiled=True): levels[l] (R,H,W,ceil(H2s[l]/8),W2s[l]/8,8,8),
 * edge e's volume at row slot[e] (slot null: row e), coords (E,H,W,2) f32 ->
 * out (E, num_levels*49, H, W) fp16, bit-exact with droid_corr_pyramid_lookup
 * on the row-major volume.  W2s[l] % 8 == 0, 16-B aligned levels. */
int droid_corr_pyramid_lookup_tiled(const void* const* levels, const int* H2s, const int* W2s, const int* slot,
                                    int num_levels, const float* coords, void* out, int E, int H, int W,
                                    hipStream_t stream);

/* CorrBlock lookup (fp16, r=3, 4 levels) writing channels-last rows
 * out (E,H,W,out_cstride) with zeros past channel 196: the A operand of the
 * fused update operator's first (1x1) conv. */
int droid_corr_pyramid_lookup_nhwc(const void* const* levels, const int* H2s, const int* W2s,
                                   int num_levels, const float* coords, void* out, int out_cstride,
                                   int E, int H, int W, hipStream_t stream);


/* CorrBlock pyramid construction (modules/corr.py:24-38,63-71) for E edges in
 * one pass: fmaps (NF,H,W,128) fp16 = frame features / 4 in NHWC (the
 * AltCorrBlock level 0), f1/f2 (E) int32 query / target frames; level l =
 * avgpool^l(<fmaps[f1[e]], fmaps[f2[e]]>) in fp16 (fp32-accumulated GEMM,
 * float-sum/4 pooling as F.avg_pool2d) written to levels[l] as
 * (E,H,W,ceil(H_l/8),W_l/8,8,8) 8x8 tiles when tiled (W % 64 == 0) or
 * (E,H,W,H_l,W_l).  H, W multiples of 8. */
int droid_corr_volume_pyramid(const void* fmaps, const int* f1, const int* f2, int E, int NF, int H, int W,
                              void* const* levels, int tiled, hipStream_t stream);

/* CorrBlock lookup fused with the update operator's corr_encoder[0]
 * (modules/corr.py:40-50 + droid_net.py:84-86): out (E,H,W,128) fp16 =
 * relu(conv1x1(lookup(coords), w) + bias), the 196-channel lookup never
 * leaving the CU (bit-identical to droid_corr_pyramid_lookup_nhwc's values).
 * levels: the 4 fp16 volumes (E,H,W,H2,W2); coords
 * (E,H,W,2) f32; w [128][224] fp16 (channel-major rows, columns >= 196 zero);
 * bias [128] f32.  Needs H*W % 128 == 0, else DROID_UNSUPPORTED. */
int droid_corr_lookup_ce0(const void* const* levels, const int* H2s, const int* W2s, const float* coords,
                          const void* w, const float* bias, void* out, int E, int H, int W, hipStream_t stream);

/* droid_corr_lookup_ce0 on volumes stored in 8x8 tiles: level l is
 * (E,H,W,ceil(H2/8),W2/8,8,8) fp16 - element (y,x) of a slice at
 * ((y/8)*(W2/8) + x/8)*64 + (y%8)*8 + x%8, rows past H2 unused - so the 8
 * window rows of a lookup touch ~3.5 128-B lines instead of 8.  The
 * layout is internal to this build (CorrBlock(tiled=True) writes it in
 * add_factors); results are bit-identical to droid_corr_lookup_ce0 on the
 * reference layout.  Needs W2 % 8 == 0 on every level. */
int droid_corr_lookup_ce0_tiled(const void* const* levels, const int* H2s, const int* W2s, const float* coords,
                                const void* w, const float* bias, void* out, int E, int H, int W,
                                hipStream_t stream);
/* droid_corr_lookup_ce0_tiled on a slot pool: the levels hold R >= E edge
 * volumes and edge e's is row slot[e] (device int32 (E), every entry in
 * [0, R)).  The frontend's edge edits (factor_graph.py:85-160) then append and
 * drop volumes by slot instead of copying the whole pyramid. */
int droid_corr_lookup_ce0_tiled_slots(const void* const* levels, const int* H2s, const int* W2s, const int* slot,
                                      const float* coords, const void* w, const float* bias, void* out, int E,
                                      int H, int W, hipStream_t stream);

/* The same lookup + corr_encoder[0] computed WITHOUT the volume: the 4
 * correlation levels are formed on demand on MFMA from a feature pyramid
 * pyr[l] (NF,H_l,W_l,128) fp16 = avgpool^l(fmap/4) (the reference's
 * AltCorrBlock pyramid, corr.py:91-104): per 8x8 query tile the union of the
 * windows is multiplied against the query features, rounded to fp16 and read
 * with the volume lookup's bilinear arithmetic.  f1/f2 (E) int32: pyramid row
 * of each edge's query / target features; coords (E,H,W,2) f32; w, bias as
 * droid_corr_lookup_ce0.  Needs H % 8 == 0 and W % 8 == 0. */
int droid_corr_alt_ce0(const void* const* pyr, const int* Hl, const int* Wl, const int* f1, const int* f2,
                       const float* coords, const void* w, const float* bias, void* out, int E, int H, int W,
                       hipStream_t stream);

/* droid_corr_alt_ce0 with the edges walked in `order` (device int32, a
 * permutation of 0..E-1; null = edge order): grouping edges that share a
 * target frame keeps its pyramid rows in L2 across their tiles.  Outputs are
 * identical for any order. */
int droid_corr_alt_ce0_ordered(const void* const* pyr, const int* Hl, const int* Wl, const int* f1, const int* f2,
                               const int* order, const float* coords, const void* w, const float* bias, void* out,
                               int E, int H, int W, hipStream_t stream);

/* ---- update operator ----------------------------------------------------
 * Implicit-GEMM convolution on MFMA (UpdateModule / ConvGRU convs,
 * droid_net.py:78-143, modules/gru.py:19-32), NHWC fp16 in, fp32 accumulate.
 * Input = channel concatenation of nsrc (<=4) NHWC sources (C[s] channels at
 * pixel stride cstride[s], multiples of 8); wp = packed weights
 * [Cout][nstage][64] fp16 (droid_mi355x.fused.pack_conv: nstage = ks*ks*sum_s ceil(C_s/64),
 * or ceil(ks*ks/8) for one 8-channel source); ks odd <= 7, "same" padding.
 * epi: 0 = act(acc + bias + bbias[b]) (act 0 none / 1 relu) -> out fp16 slice;
 *      1 = GRU z|r gates (sigmoid; z -> zout, r*h -> rnet);
 *      2 = GRU update  h' = (1-z) h + z tanh(.) -> out;
 *      3 = heads: out32 fp32, channels >= 2 through sigmoid;
 *      4 = GRU global context: mean over pixels of sigmoid(.)*h added into out32[b][co]. */
int droid_conv_nhwc_f16(const void* const* srcs, const int* C, const int* cstride, int nsrc,
                        const void* wp, const float* bias, const float* bbias, int B, int H, int W,
                        int Cout, int ks, int act, int epi, void* out, int out_cstride, int out_coff,
                        const void* h, int h_cstride, const void* z, int z_cstride, void* zout,
                        void* rnet, int gru_ch, void* out32, hipStream_t stream);

/* ConvGRU z|r and q gates (modules/gru.py:19-32) with the context-feature term
 * factored out per source frame: the gate argument is conv3x3(srcs) (the srcs
 * exclude inp) + bias + bbias[b] + pre[pre_idx[b], y, x, pre_coff + co], where
 * pre (frames,H,W,pre_cstride) fp16 holds conv3x3(inp[frame]) with the inp
 * columns of the gate weights - identical for every edge leaving that frame.
 * epi is 1 (z|r gates, Cout 256) or 2 (GRU update, Cout 128); the other
 * arguments as droid_conv_nhwc_f16 (ks 3, no act).  Runs on the band tiles
 * only (W in {16,32,64}, H*W % 256 == 0 for z|r, % 384 for q), else returns
 * DROID_UNSUPPORTED. */
int droid_conv_gru_pre_f16(const void* const* srcs, const int* C, const int* cstride, int nsrc,
                           const void* wp, const float* bias, const float* bbias, int B, int H, int W,
                           int Cout, int epi, void* out, int out_cstride, int out_coff, const void* h,
                           int h_cstride, const void* z, int z_cstride, void* zout, void* rnet, int gru_ch,
                           const void* pre, const long long* pre_idx, int pre_cstride, int pre_coff,
                           hipStream_t stream);

/* The same 3x3 convs as Winograd F(2,3) along x (2/3 of the direct conv's
 * multiplies; the reference runs them through cuDNN under autocast,
 * droid_net.py:84-103, modules/gru.py:19-32).  wt = weights transformed by
 * droid_mi355x.fused.pack_conv_wino ([6*chunks][4][Cout][32] fp16); epi 0 (act
 * 0 / 1 -> out) or, with pre / pre_idx / pre_cstride / pre_coff as in
 * droid_conv_gru_pre_f16, 1 (z|r gates) / 2 (GRU update).  Needs W == 64,
 * H % 4 == 0, Cout % 128 == 0, else returns DROID_UNSUPPORTED so the caller
 * runs the direct conv.  Measured slower than droid_conv_nhwc_f16 /
 * droid_conv_gru_pre_f16 on MI355X (issue-bound; see conv_wino_kernel): the
 * update operator uses it only when DROID_CONV_WINO=1. */
int droid_conv_wino_f16(const void* const* srcs, const int* C, const int* cstride, int nsrc, const void* wt,
                        const float* bias, const float* bbias, int B, int H, int W, int Cout, int act, int epi,
                        void* out, int out_cstride, int out_coff, const void* h, int h_cstride, const void* z,
                        int z_cstride, void* zout, void* rnet, int gru_ch, const void* pre,
                        const long long* pre_idx, int pre_cstride, int pre_coff, hipStream_t stream);

/* Batched fp16 transpose (the reference-layout drop-in's NCHW <-> NHWC state
 * conversions, droid_net.py:111-143 hands the operator NCHW tensors):
 * dst[b][c][r] = src[b][r][c] for r < R, 0 for R <= r < ldd; src (B,R,C) and
 * dst (B,C,ldd) fp16 contiguous.  NCHW -> NHWC: R = channels, C = H*W (ldd > R
 * zero-pads the channels); NHWC -> NCHW: R = H*W, C = channels. */
int droid_transpose_f16(const void* src, void* dst, int B, int R, int C, int ldd, hipStream_t stream);

/* corr_encoder[0] (droid_net.py:84-86: 1x1 conv 196 -> 128, bias, ReLU) read
 * straight from the reference's NCHW lookup (modules/corr.py:40-50 returns
 * (1, E, 196, H, W)): src (E, C, HW) fp16, w [128][K] fp16 (K % 32 == 0, K >= C,
 * columns >= C zero), bias [128] f32 -> out (E, HW, 128) fp16 = act(w . src +
 * bias), act = ReLU when relu != 0.  The reference-layout drop-in's path (no
 * channels-last copy of the lookup).  Needs HW % 128 == 0, C <= 256. */
int droid_conv1x1_nchw_f16(const void* src, int C, const void* w, int K, const float* bias, void* out, int E,
                           int HW, int relu, hipStream_t stream);

/* UpdateModule delta/weight heads fused (droid_net.py:95-103, 132-133): conv3x3
 * srcs -> 256 (wp, bias, ReLU; the delta.0 || weight.0 hidden map) feeding the
 * block-diagonal conv3x3 256 -> 4 (hw [48][256] fp16, row = tap*4 + c, tap =
 * ky*3 + kx, rows 36..47 zero) without writing the hidden map; raw head sums
 * (no head bias, no sigmoid) are atomically added into out32 (B,H,W,4) fp32,
 * which the caller zeroes.  Needs W in {16,32,64} and H*W % 256 == 0, else
 * returns DROID_UNSUPPORTED. */
int droid_conv_dw_head_f16(const void* const* srcs, const int* C, const int* cstride, int nsrc, const void* wp,
                           const float* bias, int B, int H, int W, const void* hw, void* out32,
                           hipStream_t stream);

/* flow_encoder[0] (droid_net.py:88-90): out (E,H,W,128) fp16 = relu(conv7x7(motn)
 * + bias) from the motion features motn (E,4,H,W) f32 (cast to fp16 as under
 * autocast); w [128][416] fp16 with column t*8 + c = weight[co][c][t/7][t%7]
 * for taps t < 49 and channels c < 4, zero elsewhere.  Needs W in
 * {16,32,64,128} and H*W % 128 == 0. */
int droid_flow_enc0_f16(const float* motn, const void* w, const float* bias, void* out, int E, int H, int W,
                        hipStream_t stream);

/* ConvGRU global context (modules/gru.py:19-32): glo[e][co] = mean over the
 * H*W pixels of edge e of sigmoid(w . h + bias)[co] * h[co], for h (E,H,W,128)
 * fp16 and the 1x1 conv w [128][128] fp16 ([co][ci]), bias [128] f32 -> glo
 * (E,128) f32 (plain stores, deterministic).  Needs H*W % 64 == 0. */
int droid_gru_global_f16(const void* h, const void* w, const float* bias, float* glo, int E, int HW,
                         hipStream_t stream);
/* the same split into `splits` pixel ranges per edge (more workgroups than a
 * small graph has edges): part (splits,E,128) f32, range y = its share of the
 * mean; glo = part summed over the ranges in order */
int droid_gru_global_split_f16(const void* h, const void* w, const float* bias, float* part, int splits,
                               int E, int HW, hipStream_t stream);

/* The heads' finish (droid_net.py:128-132, factor_graph.py:209-211): head
 * (E,HW,4) f32 raw head sums [du, dv, wu, wv] of droid_conv_dw_head_f16, b [4]
 * f32 -> target (E,HW,2) = base + head[0:2] + b[0:2] (base (E,HW,2) f32 or
 * null: delta), weight (E,HW,2) = sigmoid(head[2:4] + b[2:4]); when target_ba
 * and weight_ba are given, also both maps in the BA's (rows,2,HW) layout at
 * rows row0 + e (droid_ba's targets / weights). */
int droid_head_finish_f32(const float* head, const float* b, const float* base, float* target, float* weight,
                          float* target_ba, float* weight_ba, int row0, int E, int HW, hipStream_t stream);

/* GraphAgg's damping into the BA (droid_net.py:73, factor_graph.py:211,221):
 * for k < nba, frame frames[k], map[k] = its row of er (U,HW) fp16 (the raw
 * eta conv output) or -1: state (N,HW) f32 [frame] = 0.01 softplus(er[map])
 * where map >= 0, out (nba,HW) f32 [k] = 0.2 state[frame] + ep. */
int droid_eta_damping_f32(const void* er, const int* map, const int* frames, float* state, float* out, int nba,
                          int HW, float ep, hipStream_t stream);

/* the ConvGRU's global gate terms (gru.py:29-32: convz_glo | convr_glo | convq_glo
 * on glo): b + glo w^T, written as out_zr (E,256) f32 = the z | r terms and
 * out_q (E,128) f32 = the q terms (the two gate convs' per-image biases);
 * glo = sum over `splits` of part (splits,E,128) f32 (the in-order sum of
 * droid_gru_global_split_f16's ranges; splits = 1 for droid_gru_global_f16's
 * output), w (384,128) f32 row-major, 16-B aligned. */
int droid_glo_gates_f32(const float* part, int splits, const float* w, const float* b, float* out_zr, float* out_q,
                        int E, hipStream_t stream);

/* GraphAgg scatter_mean (droid_net.py:27-45, torch_scatter.scatter_mean over
 * dim 1): out[u] = mean of src rows seg_idx[seg_ptr[u] .. seg_ptr[u+1]), rows of
 * `row` fp16 values (row % 8 == 0), fp32 accumulation.  seg_ptr (U+1), seg_idx
 * (E) int64: the edges grouped by source frame (CSR of `inverse`). */
int droid_segment_mean_f16(const void* src, const int64_t* seg_ptr, const int64_t* seg_idx, void* out,
                           int num_segments, long row, hipStream_t stream);

/* replaces altcorr_forward (src/droid.cpp:193-203, altcorr_kernel.cu:290-319)
 * fmap1 (B,H,W,C), fmap2 (B,H2,W2,C) dtype (f16|f32), coords (B,S,H,W,2) f32
 * -> corr (B,S,(2r+1)^2,H,W) dtype.  radius must be 3. */
int droid_altcorr_forward(int dtype, const void* fmap1, const void* fmap2, const float* coords,
                          void* corr, int B, int S, int H, int W, int H2, int W2, int C, int radius,
                          hipStream_t stream);

/* replaces altcorr_backward (src/droid.cpp:205-217, altcorr_kernel.cu:321-356), f32 only.
 * fmap1_grad/fmap2_grad must be zero-initialised; coords grad is identically 0. */
int droid_altcorr_backward(const float* fmap1, const float* fmap2, const float* coords,
                           const float* corr_grad, float* fmap1_grad, float* fmap2_grad, int B,
                           int S, int H, int W, int H2, int W2, int C, int radius,
                           hipStream_t stream);

/* ---- geometry ----------------------------------------------------------- */

/* DepthVideo.reproject -> pops.projective_transform (depth_video.py:139-147,
 * projective_ops.py:96-125), optionally fused with the update() motion
 * features (factor_graph.py:202-204):
 * poses (N,7), disps (N,H,W), intrinsics (N,4), ii/jj (E) int64
 * -> coords (E,H,W,2), valid (E,H,W) [nullable],
 *    motn (E,4,H,W) = clamp([coords-grid, target-coords], +-64) [nullable; needs target (E,H,W,2)]. */
int droid_projective_transform(const float* poses, const float* disps, const float* intrinsics,
                               const int64_t* ii, const int64_t* jj, int E, int H, int W,
                               float* coords, float* valid, const float* target, float* motn,
                               hipStream_t stream);

/* replaces frame_distance (src/droid.cpp:120-136, droid_kernels.cu:1438-1460) -> dist (E) */
int droid_frame_distance(const float* poses, const float* disps, const float* intrinsics,
                         const int64_t* ii, const int64_t* jj, int E, int H, int W, float beta,
                         float* dist, hipStream_t stream);

/* FactorGraph.add_proximity_factors after the distances (factor_graph.py:305-369;
 * the reference walks it in Python - no droid_backends export exists for it):
 * d = the (t-t0) x (t-t1) distances of video.distance over the meshgrid
 * [t0,t) x [t1,t), row-major; ei/ej (ne) int32 = ii|ii_bad|ii_inac, jj|...;
 * n_cap = candidate pairs that may still be accepted before the edge list
 * exceeds max_factors.  -> out_i/out_j (n_cap) int32 accepted pairs in
 * acceptance order, *out_count (all device).  The caller adds the static
 * neighbour edges (and their (j, i) twins) itself.  ws: droid_proximity_workspace bytes. */
size_t droid_proximity_workspace(int t0, int t1, int t);
int droid_proximity_select(const float* d, int t0, int t1, int t, int rad, int nms, float thresh,
                           const int* ei, const int* ej, int ne, int stereo, int n_cap, int* out_i,
                           int* out_j, int* out_count, void* ws, size_t ws_bytes, hipStream_t stream);

/* MotionFilter feature encoder (modules/extractor.py BasicEncoder, norm_fn
 * 'instance' = fnet): nn.InstanceNorm2d(affine=False) of an NHWC fp16 map
 * (N, HW, C), fused with the ReLU / residual add around it.  mode 0 relu(n(x)),
 * 1 relu(res + relu(n(x))), 2 relu(n(x) + res), 3 n(x).  C % 8 == 0, C <= 512;
 * out may be x.  ws: droid_instance_norm_workspace bytes. */
size_t droid_instance_norm_workspace(int N, int HW, int C);
int droid_instance_norm_act_f16(const void* x, const void* res, void* out, int N, int HW, int C, int mode,
                                float eps, void* ws, size_t ws_bytes, hipStream_t stream);

/* replaces projmap (src/droid.cpp:139-154, droid_kernels.cu:1463-1488)
 * -> coords (E,H,W,3), valid (E,H,W,1) */
int droid_projmap(const float* poses, const float* disps, const float* intrinsics,
                  const int64_t* ii, const int64_t* jj, int E, int H, int W, float* coords,
                  float* valid, hipStream_t stream);

/* replaces iproj (src/droid.cpp:157-166, droid_kernels.cu:1518-1541) -> points (N,H,W,3) */
int droid_iproj(const float* poses, const float* disps, const float* intrinsics, int N, int H,
                int W, float* points, hipStream_t stream);

/* replaces depth_filter (src/droid.cpp:220-234, droid_kernels.cu:1491-1515)
 * ix (n) int64, thresh (n) f32, disps (num,H,W) -> counter (n,H,W) */
int droid_depth_filter(const float* poses, const float* disps, const float* intrinsics,
                       const int64_t* ix, const float* thresh, int n, int num, int H, int W,
                       float* counter, hipStream_t stream);

/* ---- dense bundle adjustment -------------------------------------------
 * replaces ba (src/droid.cpp:88-117 -> ba_cuda droid_kernels.cu:1314-1434).
 *
 * A plan captures everything of one ba() call that depends only on the edge
 * list (kx = unique([t0,t1) U ii), per-frame edge lists, Schur row graph, the
 * assembly lists of the reduced camera system, a fill-reducing pose order and
 * the tile-sparse structure of its Cholesky factor - SimplicialLLT's analyse
 * step, droid_kernels.cu:1192-1213).  Build it on the host from host copies of
 * ii/jj, upload it once into a caller-allocated device workspace, then run any
 * number of solves with no host synchronisation.  Frames of any out-degree are
 * accepted.  own_lo/own_hi restrict which optimised poses get a depth row on
 * this rank (edge-sharded multi-GPU BA); pass 0 / INT32_MAX for a single
 * device. */
int droid_ba_plan_create(const int64_t* ii_host, const int64_t* jj_host, int num_edges,
                         int num_frames, int ht, int wd, int t0, int t1, int eta_rows,
                         int motion_only, int own_lo, int own_hi, void** plan_out);
/* the same for one rank of an edge-sharded BA: ii/jj this rank's edges,
 * gii/gjj the global edge list the pose order and factor structure come from
 * (identical on every rank, so the reduced systems add up tile by tile) */
int droid_ba_plan_create_sharded(const int64_t* ii_host, const int64_t* jj_host, int num_edges,
                                 const int64_t* gii_host, const int64_t* gjj_host, int num_global_edges,
                                 int num_frames, int ht, int wd, int t0, int t1, int eta_rows,
                                 int motion_only, int own_lo, int own_hi, void** plan_out);
void droid_ba_plan_destroy(void* plan);
size_t droid_ba_plan_workspace_bytes(const void* plan);
/* Pose order of the plans created from now on (no reference counterpart:
 * Eigen's SimplicialLLT picks its own AMD ordering, droid_kernels.cu:1192):
 * -1 = chosen per plan by the expected dataflow makespan (default),
 * 0 identity, 1 reverse Cuthill-McKee, 2 minimum degree, 3 nested dissection.
 * Returns the previous setting, -2 for a mode outside -1..3. */
int droid_ba_set_order(int kind);
/* nb_max = largest Schur Gram tile count (16 variables) of any depth frame */
int droid_ba_plan_info(const void* plan, int* K, int* P, int* nblocks, int* nb_max);
int droid_ba_plan_kx(const void* plan, int64_t* kx_host);
/* kind 0 identity / 1 reverse Cuthill-McKee / 2 minimum degree / 3 nested
 * dissection (tile-aligned); perm[pose] =
 * elimination position (P ints); frames on the wide Schur path; tile tasks */
int droid_ba_plan_order(const void* plan, int* kind, int* perm, int* num_wide, int* ntasks);
/* The plan's packed int section (edge lists, assembly lists, task records,
 * slot map) inside the workspace: uploaded once by droid_ba_plan_upload and
 * only read afterwards (diagnostics: an integrity check of the section). */
int droid_ba_plan_ints_region(const void* plan, size_t* offset, size_t* bytes);

/* the reduced system's input tiles inside the workspace: 64x64 fp64 tiles of
 * the permuted lower triangle of A - S with the rhs as row n; the contiguous
 * region a multi-GPU caller all-reduces (SUM) between build and solve */
int droid_ba_plan_system_region(const void* plan, size_t* offset, size_t* bytes);
/* byte offset of the two int32 status words: word 0 = the last solve's, word 1
 * = the OR of the earlier solves' since droid_ba_run started or the caller
 * cleared them (sticky); bit 0 = a factorisation was not SPD (dx = 0, as the
 * reference), bit 1 = a dataflow solve timed out (that solve left poses and
 * disparities unchanged; the caller must report an error), bit 2 (with bit 1)
 * = the dataflow solve found its state corrupt: a sync counter not zeroed
 * before the launch or a task record outside the plan (also skipped) */
int droid_ba_plan_flag_offset(const void* plan, size_t* offset);
/* zero both status words, stream-ordered (start of a staged build/solve BA call) */
int droid_ba_plan_clear_status(void* plan, void* workspace, hipStream_t stream);
int droid_ba_plan_upload(void* plan, void* workspace, hipStream_t stream);

/* one GN linearisation -> reduced system in the workspace (all-reduce it here for multi-GPU) */
int droid_ba_build_system(void* plan, void* workspace, float* poses, float* disps,
                          const float* intrinsics, const float* disps_sens, const float* targets,
                          const float* weights, const float* eta, hipStream_t stream);
/* damping (diag += ep + lm*diag), fp64 Cholesky (dx = 0 on failure), back
 * substitution of dz (skipping pose t0 as the reference does), retraction of
 * poses [t0,t1) and of disps[kx] in place.  dz may be NULL when motion_only. */
int droid_ba_solve_update(void* plan, void* workspace, float* poses, float* disps,
                          const float* intrinsics, const float* disps_sens, const float* targets,
                          const float* weights, const float* eta, float lm, float ep, float* dx,
                          float* dz, hipStream_t stream);
/* droid_ba_solve_update in two steps: solve_system = damping + Cholesky (dx,
 * status word 0), apply_update = back substitution + retraction, both skipped
 * when status bit 1 (timeout) is set.  A sharded caller all-reduces (MAX) the
 * status words between them so every rank skips or applies the step alike. */
int droid_ba_solve_system(void* plan, void* workspace, float lm, float ep, float* dx, hipStream_t stream);
int droid_ba_apply_update(void* plan, void* workspace, float* poses, float* disps, const float* intrinsics,
                          const float* disps_sens, const float* targets, const float* weights,
                          const float* eta, float* dx, float* dz, hipStream_t stream);
/* `iterations` x (build_system + solve_update): droid_backends.ba on one device.
 * poses (N,7) f32, disps (N,H,W) f32 mutated in place; intrinsics (4); disps_sens (N,H,W);
 * targets/weights (E,2,H,W); eta (K or 1,H,W); dx (P,6) and dz (K,H*W) outputs. */
int droid_ba_run(void* plan, void* workspace, float* poses, float* disps, const float* intrinsics,
                 const float* disps_sens, const float* targets, const float* weights,
                 const float* eta, int iterations, float lm, float ep, float* dx, float* dz,
                 hipStream_t stream);

/* Dense damped SPD solve on the same dataflow Cholesky (every lower tile
 * present, identity order; used for direct testing and by callers with their
 * own systems).  droid_chol_set_system loads the lower triangle of A (n x n
 * fp64, row stride lda) and b (n) from device memory into the plan's tiles;
 * droid_chol_solve adds ep + lm*diag, factors and writes dx (n, fp32; zero and
 * flag bit 0 set when A is not SPD).  Upload with droid_ba_plan_upload; free
 * with droid_ba_plan_destroy. */
int droid_chol_plan_create(int n, void** plan_out);
int droid_chol_plan_info(const void* plan, int* ntasks, int* flag_offset, int* nslots, int* nslots_input);
int droid_chol_set_system(void* plan, void* workspace, const double* A, int lda, const double* b,
                          hipStream_t stream);
int droid_chol_solve(void* plan, void* workspace, float lm, float ep, float* dx, hipStream_t stream);
/* host copy of the task list (8 ints per task: type 0 POTRF 1 TRSM 2 UPDATE 3
 * BSOLVE 4 BUPD, i, j, k, a, b, 0, 0 - see csrc/ba.hpp) */
int droid_chol_plan_tasks(const void* plan, int* out);
/* tile structure of a plan's factor: slot map (nbr*nbc, -1 = zero tile), final
 * tile versions (nslots), final y versions (nbc), permuted var -> dx index (n);
 * any pointer may be NULL */
int droid_chol_plan_structure(const void* plan, int* slot, int* fin, int* ycnt, int* outmap);

#ifdef __cplusplus
}
#endif

#endif /* DROID_BACKENDS_H */
