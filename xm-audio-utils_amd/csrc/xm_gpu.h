/*
 * xm_gpu.h — the gfx950 backend's own entry points, shared between its HIP
 * translation units.  xm_shim.hip collects them (with the HIP runtime
 * wrappers) into the backend table xmh_gpu (xm_shim.h); the host C layer
 * reaches them only through that table.
 */
#ifndef XM_GPU_H
#define XM_GPU_H

#include "xm_shim.h"

#ifdef __cplusplus
extern "C" {
#endif

/* CUs of the current device (cached per device) */
int xmg_cu_count(void);
/* hipFuncAttributeMaxDynamicSharedMemorySize >= bytes for kern on the current
 * device, set once per (kernel, device) */
int xmg_func_lds(const void *kern, int bytes);

int xmg_launch_mix_fast(const XmhMixJob *j, void *stream, int *n_launches);      /* xm_resample_fast.hip */
int xmg_launch_mix_generic(const XmhMixJob *j, void *stream, int *n_launches);   /* xm_mix_generic.hip */
int xmg_launch_mix_placed(const XmhMixJob *j, void *stream, int *n_launches);
int xmg_launch_finish_s16(const int32_t *parts, int n_parts, int64_t part_stride, int64_t part_mix_stride,
                          int16_t *out, int64_t out_mix_stride, int64_t batch, int64_t samples, void *stream);
int xmg_fast_table_check(const float *H, int L, int M, int T);                   /* xm_resample_fast.hip */
/* the fused kernels' grid split (R super-periods per lane, tasks per mix for
 * S lanes per track row) and the XM_FAST_SPLIT_R test override (0: none) */
void xmg_pick_split(int64_t n_mix, int n_sp, int S, int *R_out, int *tpm_out);
int xmg_forced_split_r(void);
/* 147/320 (96k -> 44.1k): xm_resample_d2.hip; -1003 when the job is not its shape */
int xmg_launch_mix_d2(const XmhMixJob *j, void *stream, int *n_launches, int *R_out, int *tpm_out);
int xmg_d2_table_check(const float *H, int L, int M, int T);
int xmg_launch_fx_biquad(const XmhFxJob *j, void *stream);                        /* xm_fx.hip */
int xmg_launch_fx_fir(const XmhFxJob *j, void *stream);
int xmg_synth(void *out, int fmt, uint64_t seed, uint64_t clip0, int64_t n_clips, int channels, int64_t frames,
              void *stream);

#ifdef __cplusplus
}
#endif
#endif /* XM_GPU_H */
