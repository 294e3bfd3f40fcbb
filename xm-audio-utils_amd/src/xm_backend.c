/*
 * xm_backend.c — the xmh_* entry points of csrc/xm_shim.h: each forwards to
 * the backend of the calling thread's current device.  xmh_set_device(d)
 * selects the gfx950 backend (xmh_gpu, HIP device d) for d >= 0 and the host
 * CPU backend (xmh_cpu, src/cpu/) for XMH_DEV_CPU, the backend a handle was
 * created on (XmMixerConfig.n_devices == 0).  Like HIP's
 * current device the selection is per thread: every API entry point and every
 * worker of a multi-device handle sets its handle's device before any other
 * shim call.  No job ever moves between backends: a GPU handle whose device
 * is gone fails with XM_EDEVICE; it does not fall back to the CPU.
 */
#include "xm_internal.h"

static _Thread_local const XmhBackend *tls_be;   /* NULL: the GPU backend */

static inline const XmhBackend *be(void) { return tls_be ? tls_be : &xmh_gpu; }

/* HIP devices only: the CPU backend is not counted among them */
int xmh_device_count(void) { return xmh_gpu.device_count(); }

int xmh_set_device(int dev)
{
    tls_be = dev == XMH_DEV_CPU ? &xmh_cpu : &xmh_gpu;
    return tls_be->set_device(dev);
}

int xmh_malloc(void **p, size_t bytes) { return be()->malloc(p, bytes); }
void xmh_free(void *p) { be()->free(p); }
int xmh_host_alloc(void **p, size_t bytes) { return be()->host_alloc(p, bytes); }
void xmh_host_free(void *p) { be()->host_free(p); }
int xmh_stream_create(void **s) { return be()->stream_create(s); }
void xmh_stream_destroy(void *s) { be()->stream_destroy(s); }
int xmh_stream_sync(void *s) { return be()->stream_sync(s); }
int xmh_memcpy_h2d(void *dst, const void *src, size_t bytes, void *s) { return be()->memcpy_h2d(dst, src, bytes, s); }
int xmh_memcpy_d2h(void *dst, const void *src, size_t bytes, void *s) { return be()->memcpy_d2h(dst, src, bytes, s); }
int xmh_memcpy_d2d(void *dst, const void *src, size_t bytes, void *s) { return be()->memcpy_d2d(dst, src, bytes, s); }
int xmh_memset(void *dst, int v, size_t bytes, void *s) { return be()->memset(dst, v, bytes, s); }

int xmh_memcpy2d(void *dst, size_t dpitch, const void *src, size_t spitch, size_t width, size_t height, void *s)
{
    return be()->memcpy2d(dst, dpitch, src, spitch, width, height, s);
}

int xmh_event_create(void **e) { return be()->event_create(e); }
void xmh_event_destroy(void *e) { be()->event_destroy(e); }
int xmh_event_record(void *e, void *s) { return be()->event_record(e, s); }
int xmh_stream_wait(void *s, void *e) { return be()->stream_wait(s, e); }
int xmh_stream_create_cus(void **s, int lo, int hi, int *n_cus) { return be()->stream_create_cus(s, lo, hi, n_cus); }
int xmh_event_elapsed(float *ms, void *e0, void *e1) { return be()->event_elapsed(ms, e0, e1); }
int xmh_pointer_is_device(const void *p) { return be()->pointer_is_device(p); }

int xmh_memcpy_peer(void *dst, int dst_dev, const void *src, int src_dev, size_t bytes, void *s)
{
    return be()->memcpy_peer(dst, dst_dev, src, src_dev, bytes, s);
}

int xmh_comm_init_all(void **comms, int n, const int *devs) { return be()->comm_init_all(comms, n, devs); }
void xmh_comm_destroy(void *comm) { be()->comm_destroy(comm); }
int xmh_group_start(void) { return be()->group_start(); }
int xmh_group_end(void) { return be()->group_end(); }

int xmh_reduce_scatter_i32(const int32_t *send, int32_t *recv, size_t recv_count, void *comm, void *s)
{
    return be()->reduce_scatter_i32(send, recv, recv_count, comm, s);
}

int xmh_comm_check(void *comm) { return be()->comm_check(comm); }
const char *xmh_arch_name(void) { return be()->arch_name(); }

int xmh_launch_mix(const XmhMixJob *job, void *stream, int *n_launches, int *n_fast)
{
    return be()->launch_mix(job, stream, n_launches, n_fast);
}

int xmh_launch_mix_window(const XmhMixJob *job, void *stream, int *n_launches, int *n_fast)
{
    return be()->launch_mix_window(job, stream, n_launches, n_fast);
}

int xmh_launch_fx(const XmhFxJob *job, void *stream, int *n_launches) { return be()->launch_fx(job, stream, n_launches); }

int xmh_launch_mix_placed(const XmhMixJob *job, void *stream, int *n_launches)
{
    return be()->launch_mix_placed(job, stream, n_launches);
}

int xmh_launch_finish_s16(const int32_t *parts, int n_parts, int64_t part_stride, int64_t part_mix_stride,
                          int16_t *out, int64_t out_mix_stride, int64_t batch, int64_t samples, void *stream)
{
    return be()->launch_finish_s16(parts, n_parts, part_stride, part_mix_stride, out, out_mix_stride, batch, samples,
                                   stream);
}

int xmh_fast_table_check(const float *H, int L, int M, int T) { return be()->fast_table_check(H, L, M, T); }

int xmh_synth(void *out, int fmt, uint64_t seed, uint64_t clip0, int64_t n_clips, int channels, int64_t frames,
              void *stream)
{
    return be()->synth(out, fmt, seed, clip0, n_clips, channels, frames, stream);
}
