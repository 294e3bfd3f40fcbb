/*
 * xm_fake_shim.c — TEST INFRASTRUCTURE ONLY: a CPU stand-in for the HIP shim
 * (csrc/xm_shim.h), so the whole host C layer (the src/ C files: validation, staging,
 * strides, pointer tables, streaming windows, timeline placement, effects
 * chains, multi-device handles, config 5's exchange) runs under
 * AddressSanitizer and UndefinedBehaviorSanitizer on a machine without a GPU
 * (SURVEY.md §4 "fake-device backend", §5 "Sanitizers").
 *
 * It is linked only into tests/host_asan/libxm_audio_asan.so (Makefile next
 * to this file), never into the product library.
 * It stands in for the GPU backend table (xmh_gpu, csrc/xm_shim.h); the
 * product's CPU backend (src/cpu/) is linked in unchanged beside it.
 * "Device memory" is host memory; launches run the kernels' contract
 * (include/xm_audio_common.h) in plain C with the same operation order, so
 * tests/test_host_asan.py can also compare its outputs with the oracle.  Every
 * out-of-range access the host layer would hand a kernel is an ASan report
 * here.  Streams are synchronous, events record nothing.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "xm_shim.h"

#define XM_ENOMEM_ (-12)
#define XM_EINVAL_ (-22)
#define XM_ENOSYS_ (-1003)

static int fake_devices(void)
{
    const char *e = getenv("XM_FAKE_DEVICES");
    return e ? atoi(e) : 1;
}

/* failure injection for the checks: fk_set_device(dev) fails while dev == fail_dev */
static int fail_dev = -1;
__attribute__((visibility("default"))) void xm_fake_fail_device(int dev) { fail_dev = dev; }

static int fk_device_count(void) { return fake_devices(); }
static int fk_set_device(int dev) { return dev >= 0 && dev < fake_devices() && dev != fail_dev ? 0 : -1001; }

static int fk_malloc(void **p, size_t bytes)
{
    *p = malloc(bytes ? bytes : 16);
    return *p ? 0 : XM_ENOMEM_;
}

static void fk_free(void *p) { free(p); }
static int fk_host_alloc(void **p, size_t bytes) { return fk_malloc(p, bytes); }
static void fk_host_free(void *p) { free(p); }

static int fake_stream_obj;
static int fk_stream_create(void **s)
{
    *s = &fake_stream_obj;
    return 0;
}
static void fk_stream_destroy(void *s) { (void)s; }
static int fk_stream_sync(void *s)
{
    (void)s;
    return 0;
}

static int fk_memcpy_h2d(void *dst, const void *src, size_t n, void *s)
{
    (void)s;
    if (n) memmove(dst, src, n);
    return 0;
}
static int fk_memcpy_d2h(void *dst, const void *src, size_t n, void *s) { return fk_memcpy_h2d(dst, src, n, s); }
static int fk_memcpy_d2d(void *dst, const void *src, size_t n, void *s) { return fk_memcpy_h2d(dst, src, n, s); }
static int fk_memcpy_peer(void *dst, int dd, const void *src, int sd, size_t n, void *s)
{
    (void)dd;
    (void)sd;
    return fk_memcpy_h2d(dst, src, n, s);
}

static int fk_memcpy2d(void *dst, size_t dpitch, const void *src, size_t spitch, size_t width, size_t height, void *s)
{
    (void)s;
    if (!width || !height) return 0;
    if (dpitch < width || spitch < width) return XM_EINVAL_;
    for (size_t r = 0; r < height; ++r) memmove((char *)dst + r * dpitch, (const char *)src + r * spitch, width);
    return 0;
}

static int fk_memset(void *dst, int v, size_t n, void *s)
{
    (void)s;
    if (n) memset(dst, v, n);
    return 0;
}

static int fake_event_obj;
static int fk_event_create(void **e)
{
    *e = &fake_event_obj;
    return 0;
}
static void fk_event_destroy(void *e) { (void)e; }
static int fk_event_record(void *e, void *s)
{
    (void)e;
    (void)s;
    return 0;
}
static int fk_event_elapsed(float *ms, void *e0, void *e1)
{
    (void)e0;
    (void)e1;
    *ms = 0.0f;
    return 0;
}

static int fk_pointer_is_device(const void *p)
{
    (void)p;
    return 0;
}

static const char *fk_arch_name(void) { return "fake-cpu"; }

/* ---- the kernels' arithmetic contract in C (include/xm_audio_common.h) ---- */
static float gain_f32(const XmhGain *g, int64_t n)
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

static int32_t gain_q15(const XmhGain *g, int64_t n)
{
    int32_t v;
    if (g->len == 0) {
        v = n >= g->start ? g->q1 : g->q0;
    } else {
        int64_t k = n - g->start;
        k = k < 0 ? 0 : (k > g->len ? g->len : k);
        v = g->q0 + (int32_t)(((int64_t)(g->q1 - g->q0) * k) / g->len);
    }
    return (g->flags & XMH_GAIN_XFADE_OUT) ? 32768 - v : v;
}

static int16_t sat16(int32_t v) { return (int16_t)(v < -32768 ? -32768 : (v > 32767 ? 32767 : v)); }

static int32_t round_sat16(float v)
{
    float r = rintf(v);
    r = r < -32768.0f ? -32768.0f : (r > 32767.0f ? 32767.0f : r);
    return (int32_t)r;
}

static int32_t q15_term(int32_t s, int32_t g) { return (s * g + 16384) >> 15; }

static const void *track_ptr(const XmhMixJob *j, int64_t b, int tr, int elem)
{
    if (j->in_ptrs) return j->in_ptrs[b * j->n_tracks + tr];
    return (const char *)j->in + (b * j->in_mix_stride + (int64_t)tr * j->in_track_stride) * elem;
}

static void *out_ptr(const XmhMixJob *j, int64_t b, int elem)
{
    if (j->out_ptrs) return j->out_ptrs[b];
    return (char *)j->out + b * j->out_mix_stride * elem;
}

static void store(const XmhMixJob *j, int64_t b, int64_t i, int s16, int32_t acci, float accf)
{
    if (s16 && j->partial) ((int32_t *)out_ptr(j, b, 4))[i] = acci;
    else if (s16 && j->out_conv == 2) ((float *)out_ptr(j, b, 4))[i] = (float)sat16(acci) * 0x1p-15f;
    else if (s16) ((int16_t *)out_ptr(j, b, 2))[i] = sat16(acci);
    else if (j->out_conv == 1) ((int16_t *)out_ptr(j, b, 2))[i] = (int16_t)round_sat16(accf * 32768.0f);
    else ((float *)out_ptr(j, b, 4))[i] = accf + 0.0f;
}

static int fk_launch_mix(const XmhMixJob *j, void *stream, int *n_launches, int *n_fast)
{
    (void)stream;
    (void)n_fast;
    const int C = j->channels, s16 = j->fmt == 1;
    const int L = j->rs.L, M = j->rs.M, T = j->rs.T, rm = j->rs.rm;
    const int64_t N = j->frames_in;
    for (int64_t b = 0; b < j->n_mix; ++b)
        for (int64_t i = 0; i < j->frames_out; ++i) {
            const int64_t n = j->out_base + i;   /* absolute output frame */
            for (int c = 0; c < C; ++c) {
                int32_t acci = 0;
                float accf = 0.0f;
                for (int tr = 0; tr < j->n_tracks; ++tr) {
                    const void *x = track_ptr(j, b, tr, s16 ? 2 : 4);
                    float r;
                    if (L != M) {
                        const int64_t Mx = (n + rm) * M;
                        const float *h = j->rs.H + (Mx % L) * T;
                        const int64_t j0 = Mx / L - T + 1;
                        r = 0.0f;
                        for (int t = 0; t < T; ++t) {
                            const int64_t f = j0 + t;
                            float v = 0.0f;
                            if (f >= 0 && f < N)
                                v = s16 ? (float)((const int16_t *)x)[(f - j->in_base) * C + c]
                                        : ((const float *)x)[(f - j->in_base) * C + c];
                            r = r + v * h[t];
                        }
                    } else {   /* no resampling: the window holds frame n at row n - in_base */
                        const int64_t f = n - j->in_base;
                        r = s16 ? (float)((const int16_t *)x)[f * C + c] : ((const float *)x)[f * C + c];
                    }
                    if (s16) acci += q15_term(L != M ? round_sat16(r) : (int32_t)r, gain_q15(&j->gains[tr], n));
                    else accf = accf + gain_f32(&j->gains[tr], n) * r;
                }
                store(j, b, i * C + c, s16, acci, accf);
            }
        }
    if (n_launches) *n_launches += 1;
    return 0;
}

/* the fused kernel's streaming windows: not modelled here, the host falls
 * back to the generic window job */
static int fk_launch_mix_window(const XmhMixJob *j, void *stream, int *n_launches, int *n_fast)
{
    (void)j; (void)stream; (void)n_launches; (void)n_fast;
    return -1003;
}

static int fk_launch_mix_placed(const XmhMixJob *j, void *stream, int *n_launches)
{
    (void)stream;
    const int C = j->channels, s16 = j->fmt == 1;
    for (int64_t b = 0; b < j->n_mix; ++b)
        for (int64_t m = 0; m < j->frames_out; ++m)
            for (int c = 0; c < C; ++c) {
                int32_t acci = 0;
                float accf = 0.0f;
                for (int tr = 0; tr < j->n_tracks; ++tr) {
                    const int64_t tf = m - j->place[2 * tr], len = j->place[2 * tr + 1];
                    const void *xp = j->in_ptrs[b * j->n_tracks + tr];
                    const int in = tf >= 0 && tf < len;
                    if (s16) acci += q15_term(in ? ((const int16_t *)xp)[tf * C + c] : 0, gain_q15(&j->gains[tr], m));
                    else accf = accf + gain_f32(&j->gains[tr], m) * (in ? ((const float *)xp)[tf * C + c] : 0.0f);
                }
                XmhMixJob jj = *j;
                jj.partial = 0;
                store(&jj, b, m * C + c, s16, acci, accf);
            }
    if (n_launches) *n_launches += 1;
    return 0;
}

static int fk_launch_finish_s16(const int32_t *parts, int n_parts, int64_t part_stride, int64_t part_mix_stride,
                          int16_t *out, int64_t out_mix_stride, int64_t batch, int64_t samples, void *stream)
{
    (void)stream;
    for (int64_t b = 0; b < batch; ++b)
        for (int64_t i = 0; i < samples; ++i) {
            int32_t acc = 0;
            for (int q = 0; q < n_parts; ++q) acc += parts[q * part_stride + b * part_mix_stride + i];
            out[b * out_mix_stride + i] = sat16(acc);
        }
    return 0;
}

/* biquad: sosfilt order, state [clip][section][z0,z1][ch] when streaming;
 * FIR: upfirdn order, the K-1 frames before the block from hist_in */
static int fk_launch_fx(const XmhFxJob *j, void *stream, int *n_launches)
{
    (void)stream;
    const int C = j->channels;
    if (j->n_sos > 0) {
        for (int k = 0; k < j->n_clips; ++k) {
            const float *x = j->in_ptrs[k];
            float *y = j->out_ptrs[k];
            for (int c = 0; c < C; ++c) {
                float z0[64], z1[64];
                for (int s = 0; s < j->n_sos; ++s) {
                    z0[s] = j->state ? j->state[(((size_t)k * j->n_sos + s) * 2 + 0) * C + c] : 0.0f;
                    z1[s] = j->state ? j->state[(((size_t)k * j->n_sos + s) * 2 + 1) * C + c] : 0.0f;
                }
                for (int64_t n = 0; n < j->frames; ++n) {
                    float v = x[n * C + c];
                    for (int s = 0; s < j->n_sos; ++s) {
                        const float *q = j->sos + 6 * s;
                        const float o = q[0] * v + z0[s];
                        z0[s] = (q[1] * v - q[4] * o) + z1[s];
                        z1[s] = q[2] * v - q[5] * o;
                        v = o;
                    }
                    y[n * C + c] = v;
                }
                if (j->state)
                    for (int s = 0; s < j->n_sos; ++s) {
                        j->state[(((size_t)k * j->n_sos + s) * 2 + 0) * C + c] = z0[s];
                        j->state[(((size_t)k * j->n_sos + s) * 2 + 1) * C + c] = z1[s];
                    }
            }
        }
    } else if (j->fir_len > 0) {
        const int K = j->fir_len;
        if (j->hist_in && K > 1 && (!j->hist_out || j->hist_out == j->hist_in)) return XM_EINVAL_;
        for (int k = 0; k < j->n_clips; ++k) {
            const float *x = j->in_ptrs[k];
            float *y = j->out_ptrs[k];
            const size_t len = (size_t)(K - 1 + j->frames) * C;
            float *ext = malloc(sizeof(float) * (len ? len : 1));
            if (!ext) return XM_ENOMEM_;
            for (int64_t f = -(K - 1); f < j->frames; ++f)
                for (int c = 0; c < C; ++c)
                    ext[(f + K - 1) * C + c] =
                        f >= 0 ? x[f * C + c] : (j->hist_in ? j->hist_in[((int64_t)k * (K - 1) + (K - 1 + f)) * C + c] : 0.0f);
            if (j->hist_in && K > 1)
                for (int64_t i = 0; i < (int64_t)(K - 1) * C; ++i)
                    j->hist_out[(int64_t)k * (K - 1) * C + i] = ext[(j->frames) * C + i];
            for (int64_t n = 0; n < j->frames; ++n)
                for (int c = 0; c < C; ++c) {
                    float acc = 0.0f;
                    for (int t = 0; t < K; ++t) acc = acc + ext[(n + t) * C + c] * j->fir[K - 1 - t];
                    y[n * C + c] = acc;
                }
            free(ext);
        }
    } else {
        return 0;
    }
    if (n_launches) *n_launches += 1;
    return 0;
}

static int fk_fast_table_check(const float *H, int L, int M, int T)
{
    (void)H;
    (void)L;
    (void)M;
    (void)T;
    return XM_ENOSYS_;   /* no fused kernel here: every job takes the generic contract */
}

static uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static int fk_synth(void *out, int fmt, uint64_t seed, uint64_t clip0, int64_t n_clips, int channels, int64_t frames,
              void *stream)
{
    (void)stream;
    const int64_t per = frames * channels;
    for (int64_t i = 0; i < per * n_clips; ++i) {
        const uint64_t z = mix64(seed + (((clip0 + (uint64_t)(i / per)) << 32) | (uint64_t)(i % per)) *
                                            0x9E3779B97F4A7C15ULL);
        if (fmt == 2) ((float *)out)[i] = (float)((int32_t)(z >> 40) - (1 << 23)) * 0x1p-23f;
        else ((int16_t *)out)[i] = (int16_t)(uint16_t)(z >> 48);
    }
    return 0;
}

/* ---- RCCL stand-in: one rank per "device", in-process sums ----------------
 * A communicator is the address of a slot; reduce-scatter calls of one group
 * are collected and summed at group end (as RCCL's single-process group). */
typedef struct {
    const int32_t *send;
    int32_t *recv;
    size_t count;
    int rank;
} FakeRs;
static int fake_comm_n;
static int fake_comm_slot[64];
static FakeRs fake_pending[64];
static int fake_npend, fake_in_group;

static int fk_comm_init_all(void **comms, int n, const int *devs)
{
    (void)devs;
    if (n < 1 || n > 64) return -1002;
    fake_comm_n = n;
    for (int i = 0; i < n; ++i) {
        fake_comm_slot[i] = i;
        comms[i] = &fake_comm_slot[i];
    }
    return 0;
}

static void fk_comm_destroy(void *comm) { (void)comm; }

static void fake_flush(void)
{
    for (int p = 0; p < fake_npend; ++p) {
        const FakeRs *d = &fake_pending[p];
        for (size_t i = 0; i < d->count; ++i) {
            int32_t acc = 0;
            for (int q = 0; q < fake_npend; ++q) acc += fake_pending[q].send[(size_t)d->rank * d->count + i];
            d->recv[i] = acc;
        }
    }
    fake_npend = 0;
}

static int fk_group_start(void)
{
    fake_in_group = 1;
    return 0;
}

static int fk_group_end(void)
{
    fake_in_group = 0;
    if (fake_npend != fake_comm_n) return -1002;
    fake_flush();
    return 0;
}

static int fk_reduce_scatter_i32(const int32_t *send, int32_t *recv, size_t recv_count, void *comm, void *s)
{
    (void)s;
    if (!fake_in_group || fake_npend >= 64) return -1002;
    fake_pending[fake_npend++] = (FakeRs){send, recv, recv_count, *(int *)comm};
    return 0;
}

static int fk_comm_check(void *comm) { return comm ? 0 : -1002; }

static int fk_stream_wait(void *s, void *e)   /* fake launches complete in their call */
{
    (void)s;
    (void)e;
    return 0;
}

/* as if 256 CUs: the partitioned pipeline runs here too */
static int fk_stream_create_cus(void **s, int lo, int hi, int *n_cus)
{
    *n_cus = 8 * (hi - lo);
    return s ? fk_stream_create(s) : 0;
}

const XmhBackend xmh_gpu = {
    "fake-gfx950",
    fk_device_count, fk_set_device, fk_malloc, fk_free, fk_host_alloc, fk_host_free,
    fk_stream_create, fk_stream_destroy, fk_stream_sync, fk_memcpy_h2d, fk_memcpy_d2h, fk_memcpy_d2d,
    fk_memset, fk_memcpy2d, fk_event_create, fk_event_destroy, fk_event_record, fk_event_elapsed,
    fk_pointer_is_device, fk_memcpy_peer, fk_comm_init_all, fk_comm_destroy, fk_group_start, fk_group_end,
    fk_reduce_scatter_i32, fk_comm_check, fk_arch_name, fk_launch_mix, fk_launch_mix_window, fk_launch_fx,
    fk_launch_mix_placed, fk_launch_finish_s16, fk_fast_table_check, fk_synth, fk_stream_wait,
    fk_stream_create_cus,
};
