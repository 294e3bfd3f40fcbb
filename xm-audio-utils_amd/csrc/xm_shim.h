/*
 * xm_shim.h — internal C ABI between the C host layer (src/ C files) and the
 * compute backends.  Plain C types only; every hipError_t is mapped to an XM_*
 * status inside the shim (SURVEY.md §8(b) "Shim exports").
 *
 * Two backends implement it ("The CPU backend exports the
 * identical xmh_* set ... the backend is selected at create-time"):
 *   xmh_gpu  csrc/xm_shim.hip and the gfx950 kernels (HIP device ordinals >= 0);
 *   xmh_cpu  src/cpu/ — the library's own C implementation of the same jobs on
 *            the host cores (SURVEY.md §1 layer L0-cpu), selected by the device
 *            ordinal XMH_DEV_CPU (XmMixerConfig.n_devices == 0).
 * The xmh_* functions below dispatch to the backend of the calling thread's
 * current device, set by xmh_set_device() (src/xm_backend.c), the way HIP's
 * own current device is per thread; every API call sets its handle's device
 * first.  A thread that never called xmh_set_device() is on the GPU backend.
 *
 * Nothing here is public: callers use include/xm_audio_mixer.h and
 * include/xm_effects.h.
 */
#ifndef XM_SHIM_H
#define XM_SHIM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------- device gain descriptor (32 B, one per track) ------------------
 * F32: g = g0 + step * (float)k          (step precomputed on the host in fp32)
 * Q15: g = q0 + (qd * k) / len           (int64, C truncation)
 * k = clamp(n - start, 0, len); len == 0 => g = n >= start ? end : begin.
 * flags bit0: crossfade-out (g := 1 - g, Q15: 32768 - g). */
typedef struct XmhGain {
    float   g0, g1, step;     /* F32 ramp (xfade-out: g0=0, g1=1) */
    int32_t q0, q1;           /* Q15 ramp (xfade-out: 0, 32768) */
    int32_t len;              /* ramp length, < 2^24 */
    int32_t flags;            /* XMH_GAIN_* */
    int32_t pad;
    int64_t start;            /* ramp start (output frame) */
} XmhGain;                    /* 40 B */
#define XMH_GAIN_XFADE_OUT 1u

/* ---------- resampler table on the device -------------------------------- */
typedef struct XmhResample {
    int32_t L, M, T, rm;      /* L == M == 1: no resampling */
    const float *H;           /* device, L*T floats (phase-major) */
    int32_t fast;             /* 1: H equals the table baked into the 147/160 kernel */
    int32_t pad;
} XmhResample;

/* ---------- one mix job (all pointers device) ------------------------------
 * Track tr of mix b: in_ptrs ? in_ptrs[b*n_tracks+tr]
 *                            : in + (b*in_mix_stride + tr*in_track_stride) samples.
 * Output of mix b : out_ptrs ? out_ptrs[b] : out + b*out_mix_stride samples. */
typedef struct XmhMixJob {
    int32_t fmt;              /* 1 = s16, 2 = f32 */
    int32_t channels;         /* 1 or 2 */
    int32_t n_tracks;         /* 1..64 */
    int32_t n_mix;
    int64_t frames_in, frames_out;
    const void *in;
    int64_t in_track_stride, in_mix_stride;
    const void *const *in_ptrs;
    void *out;
    int64_t out_mix_stride;
    void *const *out_ptrs;
    const XmhGain *gains;     /* device, n_tracks entries */
    const XmhGain *gains_host; /* host copy (kernel-argument path), n_tracks entries */
    int32_t unity;            /* 1: every gain is constant 1.0 (pure resample fast path) */
    int32_t partial;          /* s16 only: 1 = write the int32 track sum, no saturation (config 5) */
    XmhResample rs;
    /* optional per-track effects chain (config 4): device sos table */
    const float *sos;         /* n_sos x 6, or NULL */
    int32_t n_sos;
    int32_t reserved2;
    void *scratch;            /* device scratch for staged paths */
    size_t scratch_bytes;
    /* streaming windows (xm_audio_mixer_stream_*; 0 for whole clips):
     * output row i of this launch is absolute output frame out_base + i (the
     * gain ramps see the absolute frame); input row r is absolute input frame
     * in_base + r; absolute frames outside [0, frames_in) read as zero. */
    int64_t in_base, out_base;
    /* timeline mix (xmh_launch_mix_placed): device [n_tracks][2] int64 =
     * (output frame of the track's first frame, track length in frames) */
    const int64_t *place;
    /* output format conversion in the store epilogue (XM_MIXER_OUT_CONVERT):
     * 0 none; 1 f32 mix -> s16 out = sat16(rint(y * 32768)); 2 s16 mix -> f32 out = y * 2^-15 */
    int32_t out_conv;
    /* input conversion and planar layouts (XM_MIXER_IN_CONVERT / PLANAR),
     * whole-clip jobs only (in_base = out_base = 0): XMH_IO_* bits */
    int32_t io_flags;
    /* 1: a streaming window for the fused kernel (xmh_launch_mix_window): in
     * points at the input frame of output 0 and the 32 frames before it are
     * real samples, not padding */
    int32_t window;
    /* host copy of in_ptrs (same n_mix*n_tracks device pointers), or NULL:
     * lets the launcher check a table's span for the fused kernel */
    const void *const *in_ptrs_host;
} XmhMixJob;
#define XMH_IO_IN_CONV    1   /* f32 mix reads s16 (x * 2^-15); s16 mix reads f32 (sat16(rint(x * 32768))) */
#define XMH_IO_IN_PLANAR  2   /* track = C planes of frames_in samples */
#define XMH_IO_OUT_PLANAR 4   /* mix output = C planes of frames_out samples */

/* ---------- effects job ---------------------------------------------------- */
typedef struct XmhFxJob {
    int32_t channels;
    int32_t n_clips;
    int64_t frames;
    const float *const *in_ptrs;   /* device array of n_clips device pointers */
    float *const *out_ptrs;
    const float *sos;              /* device n_sos x 6 */
    int32_t n_sos;
    int32_t fir_len;
    const float *fir;              /* device fir_len taps */
    int32_t reserved0;
    int32_t reserved;
    /* streaming state (xm_effects_process_stream; NULL for whole clips):
     * biquad: state[clip][section][z0,z1][channel], read at the start of the
     *         block and written back after its last frame;
     * FIR:    hist_in[clip][K-1][channel] = the K-1 frames before this block
     *         (replace the zero left padding); hist_out gets the K-1 frames
     *         before the next block (hist_out != hist_in). */
    float *state;
    const float *hist_in;
    float *hist_out;
} XmhFxJob;

/* ---------- runtime --------------------------------------------------------- */
int  xmh_device_count(void);
int  xmh_set_device(int dev);
int  xmh_malloc(void **p, size_t bytes);
void xmh_free(void *p);
int  xmh_host_alloc(void **p, size_t bytes);   /* pinned */
void xmh_host_free(void *p);
int  xmh_stream_create(void **s);
void xmh_stream_destroy(void *s);
int  xmh_stream_sync(void *s);
int  xmh_memcpy_h2d(void *dst, const void *src, size_t bytes, void *s);
int  xmh_memcpy_d2h(void *dst, const void *src, size_t bytes, void *s);
int  xmh_memcpy_d2d(void *dst, const void *src, size_t bytes, void *s);
int  xmh_memset(void *dst, int v, size_t bytes, void *s);
/* 2-D copy, any direction (hipMemcpyDefault): height rows of width bytes */
int  xmh_memcpy2d(void *dst, size_t dpitch, const void *src, size_t spitch, size_t width, size_t height, void *s);
int  xmh_event_create(void **e);
void xmh_event_destroy(void *e);
int  xmh_event_record(void *e, void *s);
int  xmh_event_elapsed(float *ms, void *e0, void *e1);  /* syncs e1 */
/* work enqueued on s after this call waits for the last record of e */
int  xmh_stream_wait(void *s, void *e);
/* a stream whose kernels run only on the CUs i with lo <= i % 32 < hi (a
 * partition even across the 8 XCDs for lo, hi multiples of 8); *n_cus = how
 * many CUs that is (0: no CU masks on this backend, a plain stream).  s NULL:
 * only the count */
int  xmh_stream_create_cus(void **s, int lo, int hi, int *n_cus);
int  xmh_pointer_is_device(const void *p);     /* 1 device, 0 host, <0 error */
/* device-to-device copy between (possibly different) devices, on stream s */
int  xmh_memcpy_peer(void *dst, int dst_dev, const void *src, int src_dev, size_t bytes, void *s);

/* ---------- RCCL (config 5 exchange), loaded on first use ------------------ */
/* one communicator per device of devs (distinct ordinals), ncclCommInitAll */
int  xmh_comm_init_all(void **comms, int n, const int *devs);
void xmh_comm_destroy(void *comm);
int  xmh_group_start(void);
int  xmh_group_end(void);
/* recv (recv_count int32) = block `rank` of the element-wise sum of every
 * rank's send (n * recv_count int32); enqueued on stream s */
int  xmh_reduce_scatter_i32(const int32_t *send, int32_t *recv, size_t recv_count, void *comm, void *s);
int  xmh_comm_check(void *comm);               /* XM_ECOMM on an asynchronous error */
const char *xmh_arch_name(void);

/* ---------- kernels ----------------------------------------------------------- */
/* resample (if rs.L != rs.M) + gain + ordered track sum; adds the launches
 * made to *n_launches and, if the fused 147/160 kernel took the job, 1 to
 * *n_fast (either pointer may be NULL) */
int xmh_launch_mix(const XmhMixJob *job, void *stream, int *n_launches, int *n_fast);
/* the fused kernel only, for a streaming window job (job->window = 1, or 0
 * for the window that starts at the signal's frame 0); XM_ENOSYS (-1003)
 * when the job is not its shape (the caller then runs the window through the
 * generic kernel with in_base / out_base) */
int xmh_launch_mix_window(const XmhMixJob *job, void *stream, int *n_launches, int *n_fast);
int xmh_launch_fx(const XmhFxJob *job, void *stream, int *n_launches);
/* timeline mix: out[m] = ordered sum over tracks of g_tr(m) * x_tr[m - place_tr.offset],
 * x_tr zero outside [0, place_tr.len); in_ptrs[b*n_tracks+tr] are the (resampled)
 * tracks, rs ignored */
int xmh_launch_mix_placed(const XmhMixJob *job, void *stream, int *n_launches);
/* config 5 finish: out[b][i] = sat16(sum over p of parts[p*part_stride + b*part_mix_stride + i]) */
int xmh_launch_finish_s16(const int32_t *parts, int n_parts, int64_t part_stride, int64_t part_mix_stride,
                          int16_t *out, int64_t out_mix_stride, int64_t batch, int64_t samples, void *stream);
/* 0 if the phase-major table H (L x T) equals, bit for bit, the coefficients
 * baked into the 147/160 fast kernel (tools/gen_coefs.c); -1003 otherwise */
int xmh_fast_table_check(const float *H, int L, int M, int T);
/* synthetic PCM into device memory:
 * clip c of n_clips at out + c*frames*channels samples, id = clip0 + c. */
int xmh_synth(void *out, int fmt, uint64_t seed, uint64_t clip0, int64_t n_clips,
              int channels, int64_t frames, void *stream);

/* ---------- backend table (one per backend) ------------------------------ */
typedef struct XmhBackend {
    const char *name;
    int (*device_count)(void);
    int (*set_device)(int dev);
    int (*malloc)(void **p, size_t bytes);
    void (*free)(void *p);
    int (*host_alloc)(void **p, size_t bytes);
    void (*host_free)(void *p);
    int (*stream_create)(void **s);
    void (*stream_destroy)(void *s);
    int (*stream_sync)(void *s);
    int (*memcpy_h2d)(void *dst, const void *src, size_t bytes, void *s);
    int (*memcpy_d2h)(void *dst, const void *src, size_t bytes, void *s);
    int (*memcpy_d2d)(void *dst, const void *src, size_t bytes, void *s);
    int (*memset)(void *dst, int v, size_t bytes, void *s);
    int (*memcpy2d)(void *dst, size_t dpitch, const void *src, size_t spitch, size_t width, size_t height,
                    void *s);
    int (*event_create)(void **e);
    void (*event_destroy)(void *e);
    int (*event_record)(void *e, void *s);
    int (*event_elapsed)(float *ms, void *e0, void *e1);
    int (*pointer_is_device)(const void *p);
    int (*memcpy_peer)(void *dst, int dst_dev, const void *src, int src_dev, size_t bytes, void *s);
    int (*comm_init_all)(void **comms, int n, const int *devs);
    void (*comm_destroy)(void *comm);
    int (*group_start)(void);
    int (*group_end)(void);
    int (*reduce_scatter_i32)(const int32_t *send, int32_t *recv, size_t recv_count, void *comm, void *s);
    int (*comm_check)(void *comm);
    const char *(*arch_name)(void);
    int (*launch_mix)(const XmhMixJob *job, void *stream, int *n_launches, int *n_fast);
    int (*launch_mix_window)(const XmhMixJob *job, void *stream, int *n_launches, int *n_fast);
    int (*launch_fx)(const XmhFxJob *job, void *stream, int *n_launches);
    int (*launch_mix_placed)(const XmhMixJob *job, void *stream, int *n_launches);
    int (*launch_finish_s16)(const int32_t *parts, int n_parts, int64_t part_stride, int64_t part_mix_stride,
                             int16_t *out, int64_t out_mix_stride, int64_t batch, int64_t samples, void *stream);
    int (*fast_table_check)(const float *H, int L, int M, int T);
    int (*synth)(void *out, int fmt, uint64_t seed, uint64_t clip0, int64_t n_clips, int channels, int64_t frames,
                 void *stream);
    int (*stream_wait)(void *s, void *e);
    int (*stream_create_cus)(void **s, int lo, int hi, int *n_cus);
} XmhBackend;
extern const XmhBackend xmh_gpu;   /* csrc/xm_shim.hip (tests/host_asan: a CPU stand-in) */
extern const XmhBackend xmh_cpu;   /* src/cpu/xm_cpu_backend.c */
#define XMH_DEV_CPU (-1)           /* the host CPU backend's device ordinal */

#ifdef __cplusplus
}
#endif
#endif /* XM_SHIM_H */
