/*
 * pcm.h -- C ABI of libpcm_hip.so, the MI355X (gfx950) point-set metric library.
 *
 * Drop-in boundary for 3D-FENet's loss/metric hot path.  Every entry point
 * replaces one pybind/ATen entry of the reference's vendored CUDA extensions:
 *
 *   pcm_chamfer_forward   <- chamfer_3D.forward   (metric/chamfer3D/chamfer_cuda.cpp:17-19,
 *                                                  metric/chamfer3D/chamfer3D.cu:136-154)
 *   pcm_chamfer_backward  <- chamfer_3D.backward  (metric/chamfer3D/chamfer_cuda.cpp:22-27,
 *                                                  metric/chamfer3D/chamfer3D.cu:176-195)
 *   pcm_emd_forward       <- emd.forward          (metric/emd/emd.cpp:12-17,
 *                                                  metric/emd/emd_cuda.cu:228-282)
 *   pcm_emd_backward      <- emd.backward         (metric/emd/emd.cpp:19-23,
 *                                                  metric/emd/emd_cuda.cu:302-316)
 *   pcm_icp, pcm_nearest_neighbor, pcm_best_fit_transform
 *                         <- icp / nearest_neighbor / best_fit_transform
 *                            (utils/icp.py:68-118, :49-65, :4-46; numpy + sklearn
 *                            on the host in the reference, testnet.py:62-64)
 *
 * Conventions:
 *   - all pointers are DEVICE pointers to contiguous row-major arrays:
 *     clouds [b, n, 3] float32 (AoS xyz), per-point outputs [b, n];
 *     indices are int32 like the reference's IntTensor outputs;
 *   - the caller owns every buffer (as the reference's Python wrappers do);
 *     outputs are fully written by the library (no caller zero-fill needed,
 *     except where a function says so);
 *   - work is enqueued asynchronously on `stream` (a hipStream_t; NULL = the
 *     null stream) of the CURRENT HIP device; nothing here synchronises,
 *     allocates device memory or keeps global state, so every call is
 *     reentrant and capturable into a hipGraph;
 *   - return value: PCM_OK (0) or a negative pcm_status; pcm_strerror()
 *     names it.  (The reference returned 1/0/-1 and its Python ignored it;
 *     the Python wrappers here raise RuntimeError on any non-zero status.)
 */
#ifndef PCM_H_
#define PCM_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum pcm_status {
    PCM_OK = 0,
    PCM_ERR_INVALID_ARG = -1,   /* bad shape / size / null pointer (reference: -1)  */
    PCM_ERR_LAUNCH = -2,        /* HIP launch or runtime error (reference: 0)      */
    PCM_ERR_WORKSPACE = -3,     /* workspace missing or too small                  */
    PCM_ERR_UNSUPPORTED = -4,   /* size outside what this build supports          */
    PCM_ERR_IO = -5,            /* file missing, unreadable or truncated           */
    PCM_ERR_FORMAT = -6         /* not an (npoints, 3) float .npy array            */
} pcm_status;

/* Library / ABI version: major*10000 + minor*100 + patch. */
int pcm_version(void);

/* Human-readable name of a status code (static string, never NULL). */
const char *pcm_strerror(int status);

/* ---------------------------------------------------------------------- */
/* Chamfer3D                                                               */
/* ---------------------------------------------------------------------- */

/*
 * Bidirectional nearest neighbour, squared L2 (chamfer3D.cu:12-154).
 *   dist1[b,j] = min_k ||xyz2[b,k] - xyz1[b,j]||^2 , idx1 = lowest argmin k
 *   dist2[b,k] = min_j ||xyz1[b,j] - xyz2[b,k]||^2 , idx2 = lowest argmin j
 * Distance is evaluated as fmaf(dz,dz,fmaf(dy,dy,dx*dx)), dx = target - query.
 * Non-finite inputs follow the reference's 512-point tile semantics exactly.
 * m == 0 leaves dist1/idx1 untouched, n == 0 leaves dist2/idx2 untouched
 * (as the reference's loops do).  b, n, m >= 0.
 */
int pcm_chamfer_forward(const float *xyz1, const float *xyz2, int b, int n, int m,
                        float *dist1, float *dist2, int32_t *idx1, int32_t *idx2,
                        void *stream);

/*
 * Fused forward + loss (extension; replaces the torch reductions that
 * loss/loss.py:34-36 and utils/metrics.py:56-60 run on the forward's outputs):
 * everything pcm_chamfer_forward does, plus
 *   mean_out[0] = mean(dist1), mean_out[1] = mean(dist2)   (device float[2])
 * summed in a fixed order (deterministic run to run).  Needs b, n, m > 0 and a
 * device workspace of pcm_chamfer_workspace_bytes(b, n, m) bytes that is
 * ZERO-FILLED when first allocated; the kernels keep it consistent across
 * stream-ordered calls (not concurrent ones), so it is zero-filled only once.
 */
size_t pcm_chamfer_workspace_bytes(int b, int n, int m);
int pcm_chamfer_forward_loss(const float *xyz1, const float *xyz2, int b, int n, int m,
                             float *dist1, float *dist2, int32_t *idx1, int32_t *idx2,
                             float *mean_out, void *workspace, size_t workspace_bytes,
                             void *stream);

/*
 * Fused Chamfer loss + gradient (extension): the training step of
 * loss/loss.py:31-37 (chamfer_3DDist forward + torch.mean(dist1) +
 * torch.mean(dist2)) and its backward (chamfer3D.cu:155-195) in ONE launch:
 *   - everything pcm_chamfer_forward does (dist1, dist2, idx1, idx2);
 *   - mean_out[0] = mean(dist1), mean_out[1] = mean(dist2),
 *     mean_out[2] = mean_out[0] + mean_out[1]        (device float[3]);
 *   - gradxyz1/gradxyz2 = gradients of  w1*sum(dist1) + w2*sum(dist2),
 *     bit-identical to pcm_chamfer_backward with graddist1 = w1 and
 *     graddist2 = w2 everywhere (w1 = 1/(b*n), w2 = 1/(b*m) for the mean loss).
 * Deterministic.  Needs b > 0, 0 < n, m <= 1024 (else PCM_ERR_UNSUPPORTED:
 * use pcm_chamfer_forward_loss + pcm_chamfer_backward) and the zero-filled
 * workspace of pcm_chamfer_workspace_bytes(b, n, m) (the same buffer serves
 * pcm_chamfer_forward_loss; stream-ordered reuse only).
 */
int pcm_chamfer_loss_grad(const float *xyz1, const float *xyz2, int b, int n, int m, float w1, float w2,
                          float *dist1, float *dist2, int32_t *idx1, int32_t *idx2, float *mean_out,
                          float *gradxyz1, float *gradxyz2, void *workspace, size_t workspace_bytes,
                          void *stream);

/*
 * The fused loss + gradient as train.py:163-176 drives it (extension):
 *   chamfer_loss = mean(dist1) + mean(dist2) on fake.transpose(2, 1), then
 *   total_loss = chamfer_loss * lambda_cd + ..., total_loss.backward().
 * pcm_chamfer_loss_grad_layout is pcm_chamfer_loss_grad with
 *   - either cloud in channel planes (layout 1, as pcm_chamfer_forward_layout),
 *     read in place, its gradient written in the same layout;
 *   - grad_scale (nullable, device float): the upstream gradient the loss is
 *     expected to receive.  The gradients are those of
 *     grad_scale * (w1 sum(dist1) + w2 sum(dist2)) computed as the reference's
 *     backward does it: graddist = fl(grad_scale * w) (torch's mean backward,
 *     w = fl(1/(b n)) as torch forms it), g = 2 graddist
 *     (chamfer3D.cu:160-171).  mean_out then needs 4 floats: mean_out[3]
 *     receives the scale used.  NULL: scale 1 (pcm_chamfer_loss_grad).
 * pcm_chamfer_loss_grad_rescale is its backward once the real upstream
 * gradient *grad_loss is known (device floats; none of them may alias):
 *   - *grad_loss == *scale_used bit for bit (pass mean_out + 3): the step's
 *     gradients are already exact and the launch does nothing;
 *   - otherwise gradxyz1/2 are recomputed in place from idx1/idx2 with
 *     graddist = fl(*grad_loss * w) -- bit-identical to pcm_chamfer_backward
 *     fed that constant -- and scale_used NULL always recomputes;
 *   - *scale_next = *grad_loss (nullable): the expectation for the next step.
 * A training loop with a constant loss weight therefore recomputes once, on
 * its first step, and from then on runs the forward, the loss and the exact
 * weighted gradient in one launch plus one empty launch.  Needs 0 < n, m <=
 * 1024 and the workspace of pcm_chamfer_loss_grad.
 */
int pcm_chamfer_loss_grad_layout(const float *xyz1, const float *xyz2, int b, int n, int m, int layout1, int layout2,
                                 float w1, float w2, const float *grad_scale, float *dist1, float *dist2,
                                 int32_t *idx1, int32_t *idx2, float *mean_out, float *gradxyz1, float *gradxyz2,
                                 void *workspace, size_t workspace_bytes, void *stream);
int pcm_chamfer_loss_grad_rescale(const float *xyz1, const float *xyz2, int b, int n, int m, int layout1,
                                  int layout2, float w1, float w2, const float *grad_loss, const float *scale_used,
                                  float *scale_next, const int32_t *idx1, const int32_t *idx2, float *gradxyz1,
                                  float *gradxyz2, void *stream);
/*
 * `steps` back-to-back pcm_chamfer_loss_grad launches from one host call with
 * the arguments bound once: K steps of a native training loop on fixed
 * buffers (bench.py's N=1 region).  steps >= 0.
 */
int pcm_chamfer_loss_grad_steps(int steps, const float *xyz1, const float *xyz2, int b, int n, int m, float w1,
                                float w2, float *dist1, float *dist2, int32_t *idx1, int32_t *idx2,
                                float *mean_out, float *gradxyz1, float *gradxyz2, void *workspace,
                                size_t workspace_bytes, void *stream);

/*
 * Device-side failure of the fused-loss kernels on `workspace`: PCM_OK or
 * PCM_ERR_LAUNCH.  A gradient-phase wait of pcm_chamfer_loss_grad that times
 * out (workgroups that are not resident) is NOT a failure: the waiting
 * workgroup computes the missing argmins itself, so dist/idx/gradients are
 * exact and only time is lost.  The failure reported here is the loss poll's
 * own wait (a much longer bound) timing out: that call's means are NaN and the
 * error is sticky -- every later call on that workspace reports NaN means
 * until the caller zero-fills the workspace again (the Python wrappers detect
 * it one call later and do that, raising PcmError).  Synchronises `stream`.
 */
int pcm_chamfer_workspace_status(const void *workspace, size_t workspace_bytes, int b, int n, int m, void *stream);

/*
 * Chamfer backward (chamfer3D.cu:155-195).  With g = 2*graddist:
 *   gradxyz1[j] = g1[j](xyz1[j]-xyz2[idx1[j]]) - sum_{k: idx2[k]=j} g2[k](xyz2[k]-xyz1[j])
 *   gradxyz2[k] = g2[k](xyz2[k]-xyz1[idx2[k]]) - sum_{j: idx1[j]=k} g1[j](xyz1[j]-xyz2[k])
 * Deterministic: scatter terms are summed in ascending source index, in the
 * kernel order of the reference (gradxyz1: direct term first; gradxyz2: direct
 * term last).  gradxyz1/gradxyz2 are fully overwritten.
 */
int pcm_chamfer_backward(const float *xyz1, const float *xyz2, int b, int n, int m,
                         const float *graddist1, const float *graddist2,
                         const int32_t *idx1, const int32_t *idx2,
                         float *gradxyz1, float *gradxyz2, void *stream);

/*
 * Clouds in either layout (extension): layout 0 = [b, n, 3] rows, as above;
 * layout 1 = [b, 3, n] channel planes -- the generator's B x 3 x N output,
 * which train.py:163 hands to the loss as fake.transpose(2, 1); the
 * reference's wrapper copies such a view to rows first (dist_chamfer_3D.py:79-80),
 * these read it in place, and the backward writes each cloud's gradient in
 * that cloud's layout (so autograd's transpose backward needs no copy either).
 * Results are bit-identical to pcm_chamfer_forward / pcm_chamfer_backward on
 * the rows.  float32 only; per-point outputs and graddists stay [b, n].
 */
int pcm_chamfer_forward_layout(const float *xyz1, const float *xyz2, int b, int n, int m, int layout1, int layout2,
                               float *dist1, float *dist2, int32_t *idx1, int32_t *idx2, void *stream);
int pcm_chamfer_backward_layout(const float *xyz1, const float *xyz2, int b, int n, int m, int layout1, int layout2,
                                const float *graddist1, const float *graddist2, const int32_t *idx1,
                                const int32_t *idx2, float *gradxyz1, float *gradxyz2, void *stream);
/*
 * The layout backward with graddists read in place at any element strides
 * (batch, point) >= 0 (extension): graddist1[bi * gd1_batch_stride +
 * j * gd1_point_stride].  Strides 0 read the expanded scalar torch.mean's
 * backward hands chamfer_3DFunction.backward (loss/loss.py:36), which the
 * reference's wrapper materialised with graddist.contiguous()
 * (dist_chamfer_3D.py:59-60).  Results are bit-identical to the contiguous call.
 */
int pcm_chamfer_backward_strided(const float *xyz1, const float *xyz2, int b, int n, int m, int layout1,
                                 int layout2, const float *graddist1, long long gd1_batch_stride,
                                 long long gd1_point_stride, const float *graddist2, long long gd2_batch_stride,
                                 long long gd2_point_stride, const int32_t *idx1, const int32_t *idx2,
                                 float *gradxyz1, float *gradxyz2, void *stream);

/*
 * fp16 clouds (extension for BASELINE config 5; the reference accepted fp32
 * only).  xyz1/xyz2 hold IEEE binary16 values.  Coordinates are widened to
 * fp32 exactly, so dist/idx are bit-identical to pcm_chamfer_forward on the
 * widened clouds (fp32 outputs, as the reference's), and the gradients are the
 * fp32 path's gradients rounded once to binary16 (nearest even).
 */
int pcm_chamfer_forward_f16(const uint16_t *xyz1, const uint16_t *xyz2, int b, int n, int m,
                            float *dist1, float *dist2, int32_t *idx1, int32_t *idx2,
                            void *stream);
int pcm_chamfer_backward_f16(const uint16_t *xyz1, const uint16_t *xyz2, int b, int n, int m,
                             const float *graddist1, const float *graddist2,
                             const int32_t *idx1, const int32_t *idx2,
                             uint16_t *gradxyz1, uint16_t *gradxyz2, void *stream);

/*
 * Forward with a caller-owned workspace (extension): the same outputs as
 * pcm_chamfer_forward / pcm_chamfer_forward_f16, bit for bit.  When both
 * clouds hold >= 4096 points and b*n*m >= 2^28 it sorts them into a uniform
 * grid in the workspace and scans only the cells around each block of
 * queries (with a proof that no farther point can win, else a wider scan),
 * which is what large clouds (BASELINE config 5, N=M=16384) need; smaller
 * problems take the dense kernels and ignore the workspace.  The workspace
 * needs no initialisation and holds no state between calls.
 * pcm_chamfer_forward_ws_bytes returns 0 for a problem that takes the dense
 * kernels, so the size does not grow with the shape: a buffer shared by
 * several shapes must be sized by querying each of them (the largest answer
 * serves all); a buffer sized for a dense-path shape is too small for a grid
 * one (PCM_ERR_WORKSPACE).
 */
size_t pcm_chamfer_forward_ws_bytes(int b, int n, int m);
int pcm_chamfer_forward_ws(const float *xyz1, const float *xyz2, int b, int n, int m,
                           float *dist1, float *dist2, int32_t *idx1, int32_t *idx2,
                           void *workspace, size_t workspace_bytes, void *stream);
int pcm_chamfer_forward_ws_f16(const uint16_t *xyz1, const uint16_t *xyz2, int b, int n, int m,
                               float *dist1, float *dist2, int32_t *idx1, int32_t *idx2,
                               void *workspace, size_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------------- */
/* EMD (auction approximation)                                           */
/* ---------------------------------------------------------------------- */

/* Device workspace (bytes) pcm_emd_forward needs for a [b, n] problem. */
size_t pcm_emd_workspace_bytes(int b, int n);

/*
 * Auction-algorithm approximate EMD (emd_cuda.cu:23-282), deterministic:
 * bidders tying within the reference's 1e-6 window resolve to the lowest
 * point index (the reference lets a racing writer win).  A bidder whose best
 * value is attained by several objects bids on the one the reference's Bid
 * finds first (emd_cuda.cu:108-110, 136-139, 165-173: the lowest (thread
 * range, tile, index); the lowest index whenever n <= 2048).  Requirements as the
 * reference (emd_cuda.cu:236-249): both clouds [b, n, 3] (same n), b <= 512,
 * n % 1024 == 0 (any such n up to 2^21, else PCM_ERR_UNSUPPORTED); iters >= 1.  Outputs dist [b, n] (squared
 * distance to the assigned point) and assignment [b, n] (int32; not
 * guaranteed a bijection).  `workspace` must hold pcm_emd_workspace_bytes(b, n)
 * bytes; its content on entry is irrelevant; calls that share a workspace must
 * be stream-ordered.  `price` may be NULL; otherwise it receives the final
 * object prices [b, n] (diagnostics / parity tests).
 */
int pcm_emd_forward(const float *xyz1, const float *xyz2, int b, int n, float eps, int iters,
                    float *dist, int32_t *assignment, float *price,
                    void *workspace, size_t workspace_bytes, void *stream);

/*
 * Status of the last pcm_emd_forward on `workspace`; synchronises `stream`
 * (it reads device memory).  The auction's helper workgroups take heavy
 * iterations' full scans; a helper job whose result does not arrive within a
 * bounded wait (helpers not resident) is scanned by the batch element's own
 * workgroup instead, and no further jobs are posted in that call, so the
 * outputs never depend on residency: PCM_OK unless reading the workspace fails.
 */
int pcm_emd_workspace_status(const void *workspace, size_t workspace_bytes, int b, int n, void *stream);

/*
 * EMD backward (emd_cuda.cu:284-316): gradxyz1[j] = 2*graddist[j]*(xyz1[j] - xyz2[a[j]]).
 * The reference returns no gradient for xyz2 (emd_module.py:84-87).
 * gradxyz1 is fully overwritten.
 */
int pcm_emd_backward(const float *xyz1, const float *xyz2, int b, int n,
                     const float *graddist, const int32_t *assignment,
                     float *gradxyz1, void *stream);

/* ---------------------------------------------------------------------- */
/* ICP alignment (evaluation caller)           */
/* ---------------------------------------------------------------------- */

/*
 * Batched icp (utils/icp.py:68-118) for b independent pairs, as testnet.py:63
 * calls it per sample: A [b,n,3] (source) and B [b,n,3] (destination), float64
 * (the reference copies its inputs into float64 arrays, icp.py:89-92).
 * init_pose: NULL or [b,4,4] float64 row-major (icp.py:95-96).  Per pair:
 *   repeat: nearest neighbour of every src point in B (float64 Euclidean,
 *           lowest index on exact ties), best-fit rigid transform, src = T src,
 *   until |prev - mean(distances)| < tolerance or max_iterations passes;
 *   T_out [b,4,4] = best_fit_transform(A, src) (row-major, float64),
 *   distances [b,n] = the last pass's Euclidean NN distances (float64),
 *   iterations [b] = the reference's returned loop index i.
 * A prep launch writes B's float32 screening rows into `workspace`
 * (pcm_icp_workspace_bytes(b, n) bytes, content on entry irrelevant); then the
 * whole loop runs in one launch (each pair's source points split over K <= 16
 * workgroups, K b <= the device's CU count, so a batch of one pair still fills
 * 16 CUs).  Needs
 * max_iterations >= 1 (the reference fails otherwise), 0 < n <= 16384
 * (else PCM_ERR_UNSUPPORTED); a batch goes out in launches of at most one
 * workgroup per compute unit (K workgroups per pair, so a pair's slices are
 * resident together).  Non-finite inputs give unspecified values (the
 * reference's sklearn rejects them; the Python wrapper does the same).
 */
size_t pcm_icp_workspace_bytes(int b, int m);
int pcm_icp(const double *A, const double *B, int b, int n, const double *init_pose, int max_iterations,
            double tolerance, double *T_out, double *distances, int32_t *iterations, void *workspace,
            size_t workspace_bytes, void *stream);

/*
 * Device-side failure of the last pcm_icp on `workspace`: a pair's source
 * points are split over up to 16 workgroups that meet once per pass; a wait
 * that timed out (workgroups that could not all be resident) sets an error
 * word: PCM_ERR_LAUNCH, and the transforms are NaN.  Synchronises `stream`.
 */
int pcm_icp_workspace_status(const void *workspace, size_t workspace_bytes, int b, int n, void *stream);

/*
 * nearest_neighbor (utils/icp.py:49-65, sklearn NearestNeighbors(n_neighbors=1)):
 * for each src[b,i] (n points) the nearest dst[b,k] (m points), float64:
 *   distances[b,i] = sqrt((dx*dx + dy*dy) + dz*dz), indices[b,i] = k (int32,
 *   lowest index on exact ties).  `workspace`: pcm_icp_workspace_bytes(b, m)
 *   bytes (content on entry irrelevant).  Any m >= 1.
 */
int pcm_nearest_neighbor(const double *src, const double *dst, int b, int n, int m, double *distances,
                         int32_t *indices, void *workspace, size_t workspace_bytes, void *stream);

/*
 * best_fit_transform (utils/icp.py:4-46) for b pairs of corresponding clouds
 * A, B [b,n,3] float64: T_out [b,4,4] maps A onto B (proper rotation, the
 * reflection case fixed as icp.py:34-36 does).
 */
int pcm_best_fit_transform(const double *A, const double *B, int b, int n, double *T_out, void *stream);

/* ---------------------------------------------------------------------- */
/* Ground-truth cloud ingestion (host only)    */
/* ---------------------------------------------------------------------- */

/*
 * The reference loads each sample's ground truth with
 * np.load(data_dir_pcl + model + '/pointcloud_<numpoints>.npy')
 * (utils/datasets_old.py:37-38) and copies the collated batch to the GPU.
 * These read .npy files (format 1.0-3.0; '<f4' '>f4' '<f8' '>f8'; C or
 * Fortran order; shape (npoints, 3)) on the HOST:
 *   pcm_npy_cloud_points: *npoints = the file's row count;
 *   pcm_npy_load_clouds:  out[count, npoints, 3] float32 (host memory, e.g. a
 *     pinned staging buffer) = np.load(paths[i]).astype(float32), read by
 *     nthreads threads.  On failure returns PCM_ERR_IO / PCM_ERR_FORMAT /
 *     PCM_ERR_INVALID_ARG for the lowest failing index, stored in
 *     *failed_index (-1 on success); other slots may be partly written.
 */
int pcm_npy_cloud_points(const char *path, int *npoints);
int pcm_npy_load_clouds(const char *const *paths, int count, int npoints, float *out, int nthreads,
                        int *failed_index);

#ifdef __cplusplus
}
#endif

#endif /* PCM_H_ */
