/*
 * xm_cpu_backend.c — the host CPU backend table xmh_cpu (csrc/xm_shim.h):
 * the runtime half (memory, synchronous "streams", timestamp events) and the
 * synthetic PCM generator; the jobs are in xm_cpu_mix.c and xm_cpu_fx.c.
 * Selected per handle at create time (XmMixerConfig.n_devices == 0,
 * XmEffectsConfig.device == XM_DEVICE_CPU), never as a
 * fallback for a GPU handle.
 */
#define _POSIX_C_SOURCE 200809L
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "xm_cpu.h"

#define XM_ENOMEM_ (-12)
#define XM_EINVAL_ (-22)
#define XM_ECOMM_ (-1002)
#define XM_ENOSYS_ (-1003)

static int c_device_count(void) { return 0; }   /* not a HIP device */
static int c_set_device(int dev) { return dev == XMH_DEV_CPU ? 0 : XM_EINVAL_; }

static int c_malloc(void **p, size_t bytes)
{
    /* 64-B aligned like a device allocation (vector loads of whole lines) */
    *p = aligned_alloc(64, (bytes + 63) & ~(size_t)63);
    return *p ? 0 : XM_ENOMEM_;
}

static void c_free(void *p) { free(p); }

/* streams: every job completes inside its launch call */
static int c_stream_obj;
static int c_stream_create(void **s)
{
    *s = &c_stream_obj;
    return 0;
}
static void c_stream_destroy(void *s) { (void)s; }
static int c_stream_sync(void *s)
{
    (void)s;
    return 0;
}

/* large copies run on the pool: a host-memory batch is not one thread's worth */
typedef struct {
    char *dst;
    const char *src;
    size_t n, piece;
} CopyCtx;

static void item_copy(void *vctx, int64_t i)
{
    const CopyCtx *c = vctx;
    const size_t o = (size_t)i * c->piece, n = c->n - o < c->piece ? c->n - o : c->piece;
    memmove(c->dst + o, c->src + o, n);
}

static int c_copy(void *dst, const void *src, size_t n, void *s)
{
    (void)s;
    if (!n || dst == src) return 0;
    const size_t piece = (size_t)8 << 20;
    const char *d = dst, *sr = src;
    if (n <= piece || (d < sr + n && sr < d + n)) {   /* small, or overlapping: one memmove */
        memmove(dst, src, n);
        return 0;
    }
    CopyCtx c = {dst, src, n, piece};
    return xmc_parallel((int64_t)((n + piece - 1) / piece), item_copy, &c);
}

static int c_memset(void *dst, int v, size_t n, void *s)
{
    (void)s;
    if (n) memset(dst, v, n);
    return 0;
}

static int c_memcpy2d(void *dst, size_t dpitch, const void *src, size_t spitch, size_t width, size_t height, void *s)
{
    (void)s;
    if (!width || !height) return 0;
    if (dpitch < width || spitch < width) return XM_EINVAL_;
    for (size_t r = 0; r < height; ++r) memmove((char *)dst + r * dpitch, (const char *)src + r * spitch, width);
    return 0;
}

/* events: host timestamps (the work before a record has finished) */
typedef struct {
    struct timespec t;
} CEvent;

static int c_event_create(void **e)
{
    CEvent *ev = calloc(1, sizeof *ev);
    *e = ev;
    return ev ? 0 : XM_ENOMEM_;
}
static void c_event_destroy(void *e) { free(e); }
static int c_event_record(void *e, void *s)
{
    (void)s;
    clock_gettime(CLOCK_MONOTONIC, &((CEvent *)e)->t);
    return 0;
}
static int c_event_elapsed(float *ms, void *e0, void *e1)
{
    const struct timespec *a = &((CEvent *)e0)->t, *b = &((CEvent *)e1)->t;
    *ms = (float)((double)(b->tv_sec - a->tv_sec) * 1e3 + (double)(b->tv_nsec - a->tv_nsec) * 1e-6);
    return 0;
}

static int c_pointer_is_device(const void *p)
{
    (void)p;
    return 1;   /* host memory is this backend's device memory */
}

static int c_memcpy_peer(void *dst, int dd, const void *src, int sd, size_t n, void *s)
{
    (void)dd;
    (void)sd;
    return c_copy(dst, src, n, s);
}

/* one CPU "device": nothing to exchange with (config 5 needs GPUs) */
static int c_comm_init_all(void **comms, int n, const int *devs)
{
    (void)comms;
    (void)n;
    (void)devs;
    return XM_ECOMM_;
}
static void c_comm_destroy(void *comm) { (void)comm; }
static int c_group(void) { return XM_ECOMM_; }
static int c_reduce_scatter_i32(const int32_t *send, int32_t *recv, size_t n, void *comm, void *s)
{
    (void)send;
    (void)recv;
    (void)n;
    (void)comm;
    (void)s;
    return XM_ECOMM_;
}
static int c_comm_check(void *comm)
{
    (void)comm;
    return XM_ECOMM_;
}
static const char *c_arch_name(void) { return "cpu"; }

/* the fused kernel is a gfx950 kernel: the CPU runs every job in the general form */
static int c_launch_mix_window(const XmhMixJob *j, void *stream, int *n_launches, int *n_fast)
{
    (void)j;
    (void)stream;
    (void)n_launches;
    (void)n_fast;
    return XM_ENOSYS_;
}
static int c_fast_table_check(const float *H, int L, int M, int T)
{
    (void)H;
    (void)L;
    (void)M;
    (void)T;
    return XM_ENOSYS_;
}

/* ---- synthetic PCM (include/xm_audio_common.h xm_synth_pcm, §8(a) a11) --- */
typedef struct {
    void *out;
    int fmt, channels;
    uint64_t seed, clip0;
    int64_t frames;
} SynthCtx;

static inline uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static void item_synth(void *vctx, int64_t c)
{
    const SynthCtx *s = vctx;
    const int64_t per = s->frames * s->channels;
    const uint64_t id = (s->clip0 + (uint64_t)c) << 32;
    for (int64_t i = 0; i < per; ++i) {
        const uint64_t z = mix64(s->seed + (id | (uint64_t)i) * 0x9E3779B97F4A7C15ULL);
        if (s->fmt == 2) ((float *)s->out)[c * per + i] = (float)((int32_t)(z >> 40) - (1 << 23)) * 0x1p-23f;
        else ((int16_t *)s->out)[c * per + i] = (int16_t)(uint16_t)(z >> 48);
    }
}

int xmc_synth(void *out, int fmt, uint64_t seed, uint64_t clip0, int64_t n_clips, int channels, int64_t frames,
              void *stream)
{
    (void)stream;
    SynthCtx s = {out, fmt, channels, seed, clip0, frames};
    return xmc_parallel(n_clips, item_synth, &s);
}

/* every CPU job completes inside its call: nothing to wait for */
static int c_stream_wait(void *s, void *e)
{
    (void)s;
    (void)e;
    return 0;
}

/* no CU partitions on the host: a plain stream, and a count of 0 */
static int c_stream_create_cus(void **s, int lo, int hi, int *n_cus)
{
    (void)lo;
    (void)hi;
    *n_cus = 0;
    return s ? c_stream_create(s) : 0;
}

const XmhBackend xmh_cpu = {
    "cpu",
    c_device_count, c_set_device, c_malloc, c_free, c_malloc, c_free,
    c_stream_create, c_stream_destroy, c_stream_sync, c_copy, c_copy, c_copy,
    c_memset, c_memcpy2d, c_event_create, c_event_destroy, c_event_record, c_event_elapsed,
    c_pointer_is_device, c_memcpy_peer, c_comm_init_all, c_comm_destroy, c_group, c_group,
    c_reduce_scatter_i32, c_comm_check, c_arch_name, xmc_launch_mix, c_launch_mix_window, xmc_launch_fx,
    xmc_launch_mix_placed, xmc_launch_finish_s16, c_fast_table_check, xmc_synth, c_stream_wait,
    c_stream_create_cus,
};
