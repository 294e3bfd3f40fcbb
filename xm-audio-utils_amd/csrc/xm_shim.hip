#include <stdio.h>
#include <stdlib.h>
// xm_shim.hip — the thin C-ABI shim (SURVEY.md §1 layer L1): HIP runtime
// wrappers with every hipError_t mapped to an XM_* status, and the kernel
// dispatch for mix / effects jobs.  Only the C host layer (src/*.c) calls it.
#include <hip/hip_runtime.h>
#include <string.h>
#include "xm_shim.h"

#define XM_EDEVICE_ (-1001)
#define XM_ENOMEM_ (-12)
#define XM_ENOSYS_ (-1003)

#define map(e) map_at((e), __LINE__)
static inline int map_at(hipError_t e, int line)
{
    if (e == hipSuccess) return 0;
    if (getenv("XM_DEBUG")) fprintf(stderr, "xm_shim.hip:%d: %s\n", line, hipGetErrorString(e));
    (void)hipGetLastError();   // reported through the return code: do not leave it for a later launch check
    if (e == hipErrorOutOfMemory) return XM_ENOMEM_;
    return XM_EDEVICE_;
}

extern "C" {

int xmh_launch_mix_generic(const XmhMixJob *j, void *stream, int *n_launches);
int xmh_launch_mix_fast(const XmhMixJob *j, void *stream, int *n_launches);  // xm_resample_fast.hip
int xmh_launch_fx_biquad(const XmhFxJob *j, void *stream);
int xmh_launch_fx_fir(const XmhFxJob *j, void *stream);

int xmh_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int xmh_set_device(int dev) { return map(hipSetDevice(dev)); }

int xmh_malloc(void **p, size_t bytes)
{
    *p = nullptr;
    if (bytes == 0) bytes = 16;
    return map(hipMalloc(p, bytes));
}

void xmh_free(void *p)
{
    if (p) (void)hipFree(p);
}

int xmh_host_alloc(void **p, size_t bytes)
{
    *p = nullptr;
    return map(hipHostMalloc(p, bytes ? bytes : 16, hipHostMallocDefault));
}

void xmh_host_free(void *p)
{
    if (p) (void)hipHostFree(p);
}

int xmh_stream_create(void **s)
{
    hipStream_t h = nullptr;
    int rc = map(hipStreamCreateWithFlags(&h, hipStreamNonBlocking));
    *s = (void *)h;
    return rc;
}

void xmh_stream_destroy(void *s)
{
    if (s) (void)hipStreamDestroy((hipStream_t)s);
}

int xmh_stream_sync(void *s) { return map(hipStreamSynchronize((hipStream_t)s)); }

int xmh_memcpy_h2d(void *dst, const void *src, size_t n, void *s)
{
    return n ? map(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, (hipStream_t)s)) : 0;
}

int xmh_memcpy_d2h(void *dst, const void *src, size_t n, void *s)
{
    return n ? map(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, (hipStream_t)s)) : 0;
}

int xmh_memcpy_d2d(void *dst, const void *src, size_t n, void *s)
{
    return n ? map(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, (hipStream_t)s)) : 0;
}

int xmh_memcpy2d(void *dst, size_t dpitch, const void *src, size_t spitch, size_t width, size_t height, void *s)
{
    if (!width || !height) return 0;
    return map(hipMemcpy2DAsync(dst, dpitch, src, spitch, width, height, hipMemcpyDefault, (hipStream_t)s));
}

int xmh_memset(void *dst, int v, size_t n, void *s)
{
    return n ? map(hipMemsetAsync(dst, v, n, (hipStream_t)s)) : 0;
}

int xmh_event_create(void **e)
{
    hipEvent_t h = nullptr;
    int rc = map(hipEventCreate(&h));
    *e = (void *)h;
    return rc;
}

void xmh_event_destroy(void *e)
{
    if (e) (void)hipEventDestroy((hipEvent_t)e);
}

int xmh_event_record(void *e, void *s) { return map(hipEventRecord((hipEvent_t)e, (hipStream_t)s)); }

int xmh_event_elapsed(float *ms, void *e0, void *e1)
{
    int rc = map(hipEventSynchronize((hipEvent_t)e1));
    if (rc) return rc;
    return map(hipEventElapsedTime(ms, (hipEvent_t)e0, (hipEvent_t)e1));
}

int xmh_pointer_is_device(const void *p)
{
    hipPointerAttribute_t a;
    memset(&a, 0, sizeof a);
    hipError_t e = hipPointerGetAttributes(&a, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return 0;   // unregistered host memory
    }
    return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged ? 1 : 0;
}

const char *xmh_arch_name(void)
{
    static char name[64];
    int dev = 0;
    hipDeviceProp_t p;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&p, dev) != hipSuccess) return "none";
    strncpy(name, p.gcnArchName, sizeof name - 1);
    return name;
}

int xmh_launch_mix(const XmhMixJob *j, void *stream, int *n_launches, int *n_fast)
{
    int rc = xmh_launch_mix_fast(j, stream, n_launches);
    if (rc != XM_ENOSYS_) {   // fast path took it (or failed for real)
        if (!rc && n_fast) *n_fast += 1;
        return rc;
    }
    return xmh_launch_mix_generic(j, stream, n_launches);
}

int xmh_launch_fx(const XmhFxJob *j, void *stream, int *n_launches)
{
    int rc;
    if (j->n_sos > 0) rc = xmh_launch_fx_biquad(j, stream);
    else if (j->fir_len > 0) rc = xmh_launch_fx_fir(j, stream);
    else return 0;
    if (n_launches) *n_launches += 1;
    return rc;
}

}  // extern "C"
