#include <stdio.h>
#include <stdlib.h>
// xm_shim.hip — the thin C-ABI shim (SURVEY.md §1 layer L1): HIP runtime
// wrappers with every hipError_t mapped to an XM_* status, and the kernel
// dispatch for mix / effects jobs, collected into the gfx950 backend table
// xmh_gpu (xm_shim.h).  Only the C host layer (src/*.c) reaches it, through
// the xmh_* entry points (src/xm_backend.c).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>
#include <mutex>
#include "xm_gpu.h"

#define XM_EDEVICE_ (-1001)
#define XM_ENOMEM_ (-12)
#define XM_ENOSYS_ (-1003)
#define XM_ECOMM_ (-1002)

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

int xmg_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int xmg_set_device(int dev) { return map(hipSetDevice(dev)); }

int xmg_malloc(void **p, size_t bytes)
{
    *p = nullptr;
    if (bytes == 0) bytes = 16;
    return map(hipMalloc(p, bytes));
}

void xmg_free(void *p)
{
    if (p) (void)hipFree(p);
}

int xmg_host_alloc(void **p, size_t bytes)
{
    *p = nullptr;
    return map(hipHostMalloc(p, bytes ? bytes : 16, hipHostMallocDefault));
}

void xmg_host_free(void *p)
{
    if (p) (void)hipHostFree(p);
}

int xmg_stream_create(void **s)
{
    // a blocking stream: a handle's own stream is ordered after work the
    // caller queued on the legacy default stream (a memset or fill of the
    // output, a generator), as the caller of a synchronous call expects
    hipStream_t h = nullptr;
    int rc = map(hipStreamCreateWithFlags(&h, hipStreamDefault));
    *s = (void *)h;
    return rc;
}

void xmg_stream_destroy(void *s)
{
    if (s) (void)hipStreamDestroy((hipStream_t)s);
}

int xmg_stream_sync(void *s) { return map(hipStreamSynchronize((hipStream_t)s)); }

int xmg_memcpy_h2d(void *dst, const void *src, size_t n, void *s)
{
    return n ? map(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, (hipStream_t)s)) : 0;
}

int xmg_memcpy_d2h(void *dst, const void *src, size_t n, void *s)
{
    return n ? map(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, (hipStream_t)s)) : 0;
}

int xmg_memcpy_d2d(void *dst, const void *src, size_t n, void *s)
{
    return n ? map(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, (hipStream_t)s)) : 0;
}

}  // extern "C"

// Device-to-device rectangle copy (streaming windows: a block of every track
// appended to its window row).  hipMemcpy2DAsync's blit kernel moves these
// at ~1.5 TB/s; this one streams 16 B per lane when every pointer, pitch and
// the width are 16-B multiples (4 B otherwise), 16 KB per workgroup-row.
namespace {
constexpr int CP_THREADS = 256, CP_UNROLL = 4;
typedef int cp_v4 __attribute__((ext_vector_type(4)));
template <typename T>
__global__ __launch_bounds__(CP_THREADS) void k_copy2d(char *dst, size_t dp, const char *src, size_t sp, size_t width,
                                                       size_t height)
{
    const size_t n = width / sizeof(T);
    const size_t i0 = ((size_t)blockIdx.x * CP_UNROLL) * CP_THREADS + threadIdx.x;
    for (size_t row = blockIdx.y; row < height; row += gridDim.y) {
        const T *a = (const T *)(src + row * sp);
        T *b = (T *)(dst + row * dp);
        T v[CP_UNROLL];
#pragma unroll
        for (int u = 0; u < CP_UNROLL; ++u) {
            const size_t i = i0 + (size_t)u * CP_THREADS;
            if (i < n) v[u] = __builtin_nontemporal_load(a + i);
        }
#pragma unroll
        for (int u = 0; u < CP_UNROLL; ++u) {
            const size_t i = i0 + (size_t)u * CP_THREADS;
            if (i < n) b[i] = v[u];
        }
    }
}

bool on_device(const void *p)
{
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();   // host pointer unknown to HIP: not an error here
        return false;
    }
    return a.type == hipMemoryTypeDevice;
}
}  // namespace

extern "C" {

int xmg_memcpy2d(void *dst, size_t dpitch, const void *src, size_t spitch, size_t width, size_t height, void *s)
{
    if (!width || !height) return 0;
    const uintptr_t al = (uintptr_t)dst | (uintptr_t)src | dpitch | spitch | width;
    if ((al & 3) == 0 && width * height >= ((size_t)1 << 20) && on_device(dst) && on_device(src)) {
        const bool v16 = (al & 15) == 0;
        const size_t n = width / (v16 ? 16 : 4);
        const dim3 grid((unsigned)((n + CP_THREADS * CP_UNROLL - 1) / (CP_THREADS * CP_UNROLL)),
                        (unsigned)(height < 65535 ? height : 65535));
        if (v16)
            hipLaunchKernelGGL(k_copy2d<cp_v4>, grid, dim3(CP_THREADS), 0, (hipStream_t)s, (char *)dst, dpitch,
                               (const char *)src, spitch, width, height);
        else
            hipLaunchKernelGGL(k_copy2d<int>, grid, dim3(CP_THREADS), 0, (hipStream_t)s, (char *)dst, dpitch,
                               (const char *)src, spitch, width, height);
        return map(hipGetLastError());
    }
    return map(hipMemcpy2DAsync(dst, dpitch, src, spitch, width, height, hipMemcpyDefault, (hipStream_t)s));
}

int xmg_memset(void *dst, int v, size_t n, void *s)
{
    return n ? map(hipMemsetAsync(dst, v, n, (hipStream_t)s)) : 0;
}

int xmg_event_create(void **e)
{
    hipEvent_t h = nullptr;
    int rc = map(hipEventCreate(&h));
    *e = (void *)h;
    return rc;
}

void xmg_event_destroy(void *e)
{
    if (e) (void)hipEventDestroy((hipEvent_t)e);
}

int xmg_event_record(void *e, void *s) { return map(hipEventRecord((hipEvent_t)e, (hipStream_t)s)); }
int xmg_stream_wait(void *s, void *e) { return map(hipStreamWaitEvent((hipStream_t)s, (hipEvent_t)e, 0)); }

// CU-masked stream (config 4's pipeline: the biquad workgroups each need a
// whole CU's LDS, so the stages beside them keep to the other CUs)
int xmg_stream_create_cus(void **s, int lo, int hi, int *n_cus)
{
    const int cus = xmg_cu_count();
    uint32_t mask[64] = {};
    const int words = (cus + 31) / 32;
    int n = 0;
    for (int i = 0; i < cus && i < 64 * 32; ++i)
        if (i % 32 >= lo && i % 32 < hi) {
            mask[i / 32] |= 1u << (i % 32);
            ++n;
        }
    *n_cus = n;
    if (!s) return 0;
    *s = nullptr;
    if (n == 0 || words > 64) return -22;
    hipStream_t h = nullptr;
    const int rc = map(hipExtStreamCreateWithCUMask(&h, (uint32_t)words, mask));
    *s = (void *)h;
    return rc;
}

int xmg_event_elapsed(float *ms, void *e0, void *e1)
{
    int rc = map(hipEventSynchronize((hipEvent_t)e1));
    if (rc) return rc;
    return map(hipEventElapsedTime(ms, (hipEvent_t)e0, (hipEvent_t)e1));
}

int xmg_pointer_is_device(const void *p)
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

int xmg_memcpy_peer(void *dst, int dst_dev, const void *src, int src_dev, size_t n, void *s)
{
    if (!n) return 0;
    if (dst_dev == src_dev) return map(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, (hipStream_t)s));
    return map(hipMemcpyPeerAsync(dst, dst_dev, src, src_dev, n, (hipStream_t)s));
}

// ---- RCCL, resolved with dlopen on first use: the library has no link-time
// dependency on librccl, and a process that already loaded it (torch) shares
// that copy.  Only config 5's exchange (xm_audio_mixer_mix_spanning_s16) uses it.
}  // extern "C"
namespace {
struct Rccl {
    bool tried = false, ok = false;
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclReduceScatter) reduce_scatter = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclCommGetAsyncError) async_error = nullptr;
    decltype(&ncclGetErrorString) err_str = nullptr;
};
Rccl &rccl()
{
    static Rccl r;
    if (r.tried) return r;
    r.tried = true;
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
        if (getenv("XM_DEBUG")) fprintf(stderr, "xm_shim: librccl not found: %s\n", dlerror());
        return r;
    }
    r.init_all = (decltype(r.init_all))dlsym(h, "ncclCommInitAll");
    r.destroy = (decltype(r.destroy))dlsym(h, "ncclCommDestroy");
    r.reduce_scatter = (decltype(r.reduce_scatter))dlsym(h, "ncclReduceScatter");
    r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
    r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
    r.async_error = (decltype(r.async_error))dlsym(h, "ncclCommGetAsyncError");
    r.err_str = (decltype(r.err_str))dlsym(h, "ncclGetErrorString");
    r.ok = r.init_all && r.destroy && r.reduce_scatter && r.group_start && r.group_end && r.async_error;
    return r;
}
int cmap(ncclResult_t e, int line)
{
    if (e == ncclSuccess) return 0;
    if (getenv("XM_DEBUG"))
        fprintf(stderr, "xm_shim.hip:%d: rccl %s\n", line, rccl().err_str ? rccl().err_str(e) : "error");
    return XM_ECOMM_;
}
}  // namespace
extern "C" {

int xmg_comm_init_all(void **comms, int n, const int *devs)
{
    if (!rccl().ok) return XM_ECOMM_;
    return cmap(rccl().init_all((ncclComm_t *)comms, n, devs), __LINE__);
}

void xmg_comm_destroy(void *comm)
{
    if (comm && rccl().ok) (void)rccl().destroy((ncclComm_t)comm);
}

int xmg_group_start(void) { return rccl().ok ? cmap(rccl().group_start(), __LINE__) : XM_ECOMM_; }
int xmg_group_end(void) { return rccl().ok ? cmap(rccl().group_end(), __LINE__) : XM_ECOMM_; }

int xmg_reduce_scatter_i32(const int32_t *send, int32_t *recv, size_t recv_count, void *comm, void *s)
{
    if (!rccl().ok) return XM_ECOMM_;
    return cmap(rccl().reduce_scatter(send, recv, recv_count, ncclInt32, ncclSum, (ncclComm_t)comm, (hipStream_t)s),
                __LINE__);
}

int xmg_comm_check(void *comm)
{
    if (!rccl().ok || !comm) return XM_ECOMM_;
    ncclResult_t a = ncclSuccess;
    int rc = cmap(rccl().async_error((ncclComm_t)comm, &a), __LINE__);
    return rc ? rc : cmap(a, __LINE__);
}

// Per-device launch facts, cached (worker threads of a multi-device handle
// reach these concurrently, each on its own device).
namespace {
constexpr int XMH_MAXDEV = 64;
std::mutex g_attr_mu;
struct LdsAttr {
    const void *kern;
    int dev, bytes;
};
LdsAttr g_lds[256];
int g_n_lds = 0;
int g_cus[XMH_MAXDEV];   // 0: not read yet
}  // namespace

int xmg_cu_count(void)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= XMH_MAXDEV) return 256;
    std::lock_guard<std::mutex> g(g_attr_mu);
    if (!g_cus[dev]) {
        int c = 0;
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
        g_cus[dev] = c;
    }
    return g_cus[dev];
}

int xmg_func_lds(const void *kern, int bytes)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return XM_EDEVICE_;
    std::lock_guard<std::mutex> g(g_attr_mu);
    for (int i = 0; i < g_n_lds; ++i)
        if (g_lds[i].kern == kern && g_lds[i].dev == dev && g_lds[i].bytes >= bytes) return 0;
    const int rc = map(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
    if (rc) return rc;
    for (int i = 0; i < g_n_lds; ++i)
        if (g_lds[i].kern == kern && g_lds[i].dev == dev) {
            g_lds[i].bytes = bytes;
            return 0;
        }
    if (g_n_lds < (int)(sizeof g_lds / sizeof g_lds[0])) g_lds[g_n_lds++] = LdsAttr{kern, dev, bytes};
    return 0;
}

const char *xmg_arch_name(void)
{
    static char name[64];
    int dev = 0;
    hipDeviceProp_t p;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&p, dev) != hipSuccess) return "none";
    strncpy(name, p.gcnArchName, sizeof name - 1);
    return name;
}

int xmg_launch_mix(const XmhMixJob *j, void *stream, int *n_launches, int *n_fast)
{
    int rc = xmg_launch_mix_fast(j, stream, n_launches);
    if (rc != XM_ENOSYS_) {   // fast path took it (or failed for real)
        if (!rc && n_fast) *n_fast += 1;
        return rc;
    }
    return xmg_launch_mix_generic(j, stream, n_launches);
}

int xmg_launch_mix_window(const XmhMixJob *j, void *stream, int *n_launches, int *n_fast)
{
    const int rc = xmg_launch_mix_fast(j, stream, n_launches);
    if (!rc && n_fast) *n_fast += 1;
    return rc;
}

int xmg_launch_fx(const XmhFxJob *j, void *stream, int *n_launches)
{
    int rc;
    if (j->n_sos > 0) rc = xmg_launch_fx_biquad(j, stream);
    else if (j->fir_len > 0) rc = xmg_launch_fx_fir(j, stream);
    else return 0;
    if (n_launches) *n_launches += 1;
    return rc;
}

// host side only: clang would otherwise promote this const table to the
// device and link it against host functions there
#ifndef __HIP_DEVICE_COMPILE__
const XmhBackend xmh_gpu = {
    "gfx950",
    xmg_device_count, xmg_set_device, xmg_malloc, xmg_free, xmg_host_alloc, xmg_host_free,
    xmg_stream_create, xmg_stream_destroy, xmg_stream_sync, xmg_memcpy_h2d, xmg_memcpy_d2h, xmg_memcpy_d2d,
    xmg_memset, xmg_memcpy2d, xmg_event_create, xmg_event_destroy, xmg_event_record, xmg_event_elapsed,
    xmg_pointer_is_device, xmg_memcpy_peer, xmg_comm_init_all, xmg_comm_destroy, xmg_group_start, xmg_group_end,
    xmg_reduce_scatter_i32, xmg_comm_check, xmg_arch_name, xmg_launch_mix, xmg_launch_mix_window, xmg_launch_fx,
    xmg_launch_mix_placed, xmg_launch_finish_s16, xmg_fast_table_check, xmg_synth, xmg_stream_wait,
    xmg_stream_create_cus,
};
#endif

}  // extern "C"
