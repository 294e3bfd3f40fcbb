/*
 * xm_cpu.h — the host CPU backend (SURVEY.md §1 layer L0-cpu, §8(b): the
 * same xmh_* job set as the gfx950 kernels, selected at create time by
 * XmMixerConfig.n_devices == 0 / XM_DEVICE_CPU).  Product code: it computes
 * every job of csrc/xm_shim.h in the arithmetic of include/xm_audio_common.h
 * (separately rounded fp32 in scipy's order, Q15 integer mixing), bit for bit
 * the kernels' results, on a pool of host threads.  It shares no code with
 * oracle/ (the test-side restatement it is checked against).
 *
 * "Device memory" of this backend is host memory, streams are synchronous
 * (a job has finished when its launch returns), events are host timestamps.
 */
#ifndef XM_CPU_H
#define XM_CPU_H

#include <stddef.h>
#include <stdint.h>

#include "../../csrc/xm_shim.h"

/* ---- thread pool (xm_cpu_pool.c) ----------------------------------------
 * xmc_parallel(n, fn, ctx): fn(ctx, i) for every i in [0, n), items handed
 * out one at a time to the pool's threads and the caller; returns when all
 * are done.  Threads: XM_CPU_THREADS if set, else the CPUs of the process's
 * affinity mask (sched_getaffinity), created on first use. */
typedef void (*XmcItemFn)(void *ctx, int64_t i);
int  xmc_parallel(int64_t n, XmcItemFn fn, void *ctx);
int  xmc_threads(void);

/* ---- jobs (xm_cpu_mix.c, xm_cpu_fx.c) ------------------------------------ */
int xmc_launch_mix(const XmhMixJob *j, void *stream, int *n_launches, int *n_fast);
int xmc_launch_mix_placed(const XmhMixJob *j, void *stream, int *n_launches);
int xmc_launch_finish_s16(const int32_t *parts, int n_parts, int64_t part_stride, int64_t part_mix_stride,
                          int16_t *out, int64_t out_mix_stride, int64_t batch, int64_t samples, void *stream);
int xmc_launch_fx(const XmhFxJob *j, void *stream, int *n_launches);
int xmc_synth(void *out, int fmt, uint64_t seed, uint64_t clip0, int64_t n_clips, int channels, int64_t frames,
              void *stream);

/* ---- the contract's scalar pieces (include/xm_audio_common.h) ----------- */
static inline float xmc_gain_f32(const XmhGain *g, int64_t n)
{
    float v;
    if (g->len == 0) {
        v = n >= g->start ? g->g1 : g->g0;
    } else {
        int64_t k = n - g->start;
        k = k < 0 ? 0 : (k > g->len ? g->len : k);
        v = g->g0 + g->step * (float)(int32_t)k;
    }
    return (g->flags & XMH_GAIN_XFADE_OUT) ? 1.0f - v : v;
}

static inline int32_t xmc_gain_q15(const XmhGain *g, int64_t n)
{
    int32_t v;
    if (g->len == 0) {
        v = n >= g->start ? g->q1 : g->q0;
    } else {
        int64_t k = n - g->start;
        k = k < 0 ? 0 : (k > g->len ? g->len : k);
        v = g->q0 + (int32_t)(((int64_t)(g->q1 - g->q0) * k) / g->len);   /* C truncation */
    }
    return (g->flags & XMH_GAIN_XFADE_OUT) ? 32768 - v : v;
}

/* 1 when the gain is the same at every output frame of [n0, n1] */
static inline int xmc_gain_const(const XmhGain *g, int64_t n0, int64_t n1)
{
    if (g->len == 0) return n1 < g->start || n0 >= g->start;
    return n1 <= g->start || n0 >= g->start + g->len;
}

static inline int16_t xmc_sat16(int32_t v) { return (int16_t)(v < -32768 ? -32768 : (v > 32767 ? 32767 : v)); }

/* s16 sample from fp32: rint (ties to even, the default rounding mode), saturate */
static inline int32_t xmc_round_sat16(float v)
{
    float r = __builtin_rintf(v);
    r = r < -32768.0f ? -32768.0f : (r > 32767.0f ? 32767.0f : r);
    return (int32_t)r;
}

static inline int32_t xmc_q15_term(int32_t s, int32_t g) { return (s * g + 16384) >> 15; }

#endif /* XM_CPU_H */
