// pcm_internal.h -- tuning entry points exported by libpcm_hip.so but not part
// of the public C ABI (include/pcm.h).  Used by tools/tune_chamfer.py to A/B
// kernel variants inside one process (cdna_hip_programming.md section 5.4
// rule 24).
#pragma once
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
int pcm_tune_num_chamfer_variants(void);
int pcm_tune_chamfer_forward(int variant, const float *xyz1, const float *xyz2, int b, int n, int m,
                             float *dist1, float *dist2, int32_t *idx1, int32_t *idx2, void *stream);
int pcm_tune_chamfer_forward_layout(int variant, const float *xyz1, const float *xyz2, int b, int n, int m,
                                    int layout1, int layout2, float *dist1, float *dist2, int32_t *idx1,
                                    int32_t *idx2, void *stream);
int pcm_tune_chamfer_backward(int variant, const float *xyz1, const float *xyz2, int b, int n, int m,
                              const float *graddist1, const float *graddist2, const int32_t *idx1,
                              const int32_t *idx2, float *gradxyz1, float *gradxyz2, void *stream);
int pcm_tune_chamfer_forward_loss(int variant, int loss_mode, const float *xyz1, const float *xyz2, int b,
                                  int n, int m, float *dist1, float *dist2, int32_t *idx1, int32_t *idx2,
                                  float *mean_out, void *workspace, size_t workspace_bytes, void *stream);
int pcm_tune_num_chamfer_loss_grad_variants(void);
int pcm_tune_chamfer_loss_grad(int variant, const float *xyz1, const float *xyz2, int b, int n, int m, float w1,
                               float w2, float *dist1, float *dist2, int32_t *idx1, int32_t *idx2, float *mean_out,
                               float *gradxyz1, float *gradxyz2, void *workspace, size_t workspace_bytes,
                               void *stream);
int pcm_tune_chamfer_loss_grad_spins(unsigned wait_spins, unsigned poll_spins, const float *xyz1, const float *xyz2,
                                     int b, int n, int m, float w1, float w2, float *dist1, float *dist2,
                                     int32_t *idx1, int32_t *idx2, float *mean_out, float *gradxyz1, float *gradxyz2,
                                     void *workspace, size_t workspace_bytes, void *stream);
int pcm_tune_chamfer_slow_paths(const void *workspace, size_t workspace_bytes, int b, int n, int m, void *stream);
size_t pcm_tune_chamfer_err_offset(int which, int b, int n, int m);  // sticky error words' byte offsets
int pcm_tune_read_stamps(unsigned long long *host, int nblocks);  // profiling build only (make stamps)
int pcm_tune_num_chamfer_f16_variants(void);
int pcm_tune_chamfer_forward_f16(int variant, const uint16_t *xyz1, const uint16_t *xyz2, int b, int n, int m,
                                 float *dist1, float *dist2, int32_t *idx1, int32_t *idx2, void *stream);
// helpers: helper workgroups per batch element (-1 = default); offload_min:
// misses above which an iteration's full scans go to the helpers (-1 =
// default); diag: 1 = per-iteration counts, 2 = phase timers (csrc/emd.hip);
// wsplit: most waves a full scan is split over (1, 2, 4; <= 0 = default);
// tail_max: bidders at or below which an iteration runs in tail mode (-1 = default, 0 = never);
// spin_limit: bound of every wait between workgroups (-1 = default; 0 forces
// the timeout path: the master scans every offloaded item itself)
int pcm_tune_emd_forward_cfg(const float *xyz1, const float *xyz2, int b, int n, float eps, int iters,
                             float *dist, int32_t *assignment, float *price, void *workspace,
                             size_t workspace_bytes, int helpers, int offload_min, int diag, int wsplit,
                             int tail_max, int spin_limit, int32_t *stats, void *stream);
// batch elements of the last EMD forward whose master timed out on a helper job (>= 0)
// the grid forward (csrc/chamfer_grid.hip) at any size: mode bit 0 = binary16 clouds, bit 1 = exact scan,
// bit 2 = build kernel only, bit 3 = search kernel only; stats (nullable): 4 ints per search wave
int pcm_tune_chamfer_forward_grid(int mode, const void *xyz1, const void *xyz2, int b, int n, int m, float *dist1,
                                  float *dist2, int32_t *idx1, int32_t *idx2, void *workspace,
                                  size_t workspace_bytes, void *stream, int *stats);
// fp16 backward variant: 0 default, 1 256-target workgroups, 3 1024-target workgroups
int pcm_tune_chamfer_backward_f16(int variant, const uint16_t *xyz1, const uint16_t *xyz2, int b, int n, int m,
                                  const float *graddist1, const float *graddist2, const int32_t *idx1,
                                  const int32_t *idx2, uint16_t *gradxyz1, uint16_t *gradxyz2, void *stream);
int pcm_tune_emd_timeouts(const void *workspace, size_t workspace_bytes, int b, int n, void *stream);
#ifdef __cplusplus
}
#endif
