/*
 * xm_audio_common.h — shared types, error codes and arithmetic contract of the
 * MI355X-native xm-audio-utils PCM hot path.
 *
 * PROVENANCE.  The reference snapshot (sunyuchuan/xm-audio-utils @ 2025-03-01)
 * contains exactly one file, README.md, whose single line is "# xm-audio-utils"
 * (/root/reference/README.md:1).  It holds no header, so there is no existing
 * ABI to be compatible with.  BASELINE.json:5 fixes only the two prefixes
 * (xm_audio_mixer_*, xm_effects_*) and that the host stays in C.  Every type,
 * signature and formula below is therefore BUILD-OWNED and frozen here
 * (SURVEY.md §8(b)).  The arithmetic of the resampler, biquad and FIR is pinned
 * bit-for-bit to scipy 1.15.3 float32 resample_poly / sosfilt / upfirdn
 * (SURVEY.md §8(c)); the mixer/gain arithmetic is defined in this file.
 *
 * ARITHMETIC CONTRACT (all fp32 ops IEEE round-to-nearest-even, separately
 * rounded, no contraction, denormals preserved):
 *
 *  Resample L/M (after gcd reduction), T taps per phase, table H[L][T]:
 *    n_out = ceil(N*L/M);  for output m: Mx=(m+rm)*M, ph=Mx mod L,
 *    j_t = floor(Mx/L)-T+1+t;  acc=+0; for t=0..T-1: acc = acc + x[j_t]*H[ph][t]
 *    with x[j]=0 outside [0,N).  (scipy _signaltools.py:3686-3759, _upfirdn.py)
 *
 *  Gain ramp, evaluated at OUTPUT frame index n (both channels share it):
 *    k = clamp(n - ramp_start, 0, ramp_len)
 *    F32 : step = (gain1 - gain0) / (float)ramp_len   (fp32 divide, host side)
 *          g    = gain0 + step * (float)k              (mul, then add)
 *    Q15 : g    = gain0_q15 + ((int64)(gain1_q15 - gain0_q15) * k) / ramp_len
 *          (C division, truncates toward zero); 32768 == 1.0, range [0,65535]
 *    ramp_len == 0 : g = (n >= ramp_start) ? gain1 : gain0
 *    XM_GAIN_XFADE_OUT (crossfade A side): g = 1 - ramp(0 -> 1)
 *          F32 : g = 1.0f - (0 + (1/(float)len) * (float)k)
 *          Q15 : g = 32768 - (32768*k)/len
 *
 *  Mix, per output frame n and channel c, tracks summed in index order:
 *    F32 : acc=+0; for tr: acc = acc + g_tr[n] * r_tr[n][c]
 *    S16 : acc=0 (int32); for tr: acc += ((int32)s*g + 16384) >> 15
 *          (arithmetic shift);  out = saturate16(acc)
 *    r_tr is the track after resampling (and its effects chain, if any).
 *
 *  s16 resample: s16 -> fp32 (exact integer value) -> resample -> lrintf
 *    (ties-to-even) -> saturate to [-32768, 32767].
 */
#ifndef XM_AUDIO_COMMON_H
#define XM_AUDIO_COMMON_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#ifndef XM_API
#define XM_API __attribute__((visibility("default")))
#endif

/* ---- status codes: 0 = OK, negative = error; never errno, never exceptions */
#define XM_OK          0
#define XM_EINVAL    (-22)   /* bad argument / inconsistent sizes */
#define XM_ENOMEM    (-12)   /* host or device allocation failed */
#define XM_EDEVICE (-1001)   /* HIP runtime error or no usable GPU */
#define XM_ECOMM   (-1002)   /* RCCL / cross-device exchange failed */
#define XM_ENOSYS  (-1003)   /* feature not supported by this build */

typedef enum XmSampleFmt {
    XM_FMT_S16 = 1,          /* interleaved int16 PCM */
    XM_FMT_F32 = 2           /* interleaved float32 PCM */
} XmSampleFmt;

typedef enum XmMemKind {
    XM_MEM_HOST   = 0,       /* pointers are host memory; the call stages H2D/D2H */
    XM_MEM_DEVICE = 1        /* pointers are device (HBM) memory of cfg.device */
} XmMemKind;

typedef enum XmGainMode {
    XM_GAIN_RAMP      = 0,   /* g = ramp(gain0 -> gain1) */
    XM_GAIN_XFADE_OUT = 1    /* g = 1 - ramp(0 -> 1): crossfade source side */
} XmGainMode;

/* Per-track gain ramp (16 B of parameters per track on the device). */
typedef struct XmGainRamp {
    float   gain0, gain1;          /* F32 mixes */
    int32_t gain0_q15, gain1_q15;  /* S16 mixes, 32768 == unity, [0, 65535] */
    int64_t ramp_start;            /* output frame index where the ramp begins */
    int64_t ramp_len;              /* frames; 0 = step; must be < 2^24 */
    int32_t mode;                  /* XmGainMode */
    int32_t reserved;
} XmGainRamp;

/* Device ordinal of the host CPU backend (SURVEY.md §8(b) "n_devices (0 =
 * CPU)"): the library's own C implementation of every job, in the same
 * arithmetic as the gfx950 kernels (bit-identical results), run on the host
 * cores of the calling process (XM_CPU_THREADS threads if set, else one per
 * CPU of its affinity mask).  A mixer is created on it by
 * XmMixerConfig.n_devices == 0, an effects chain by XmEffectsConfig.device ==
 * XM_DEVICE_CPU or xm_effects_create(rate, channels, 0), synthetic PCM by
 * xm_synth_pcm(..., XM_DEVICE_CPU, NULL).  Its memory is host memory: both
 * XmMemKind values mean host pointers, used in place.  Chosen at create time
 * only: a GPU handle never falls back to it. */
#define XM_DEVICE_CPU (-1)

/* Human-readable text for a status code (static storage). */
XM_API const char *xm_strerror(int status);

/* Library version string, e.g. "xm-audio-mi355x 0.1.0 (gfx950)". */
XM_API const char *xm_version(void);

/* Number of HIP devices visible to this process (0 if none / runtime absent;
 * the CPU backend is not counted). */
XM_API int xm_device_count(void);

/* ---- rational resampler design (exported for tests and tools) ----------
 * Reduces in_rate/out_rate to L/M, designs the scipy-identical Kaiser(5)
 * windowed-sinc (2*10*max(L,M)+1 taps, fp64, cast to fp32, times L in fp32)
 * and returns the per-phase table H[L][T] (T = taps per phase).
 * If H is NULL only the sizes are returned.  H must hold L*T floats. */
typedef struct XmResampleDesign {
    int32_t L, M;          /* reduced up / down factors */
    int32_t T;             /* taps per phase */
    int32_t rm;            /* (half + pre) / M : output index offset */
    int32_t half;          /* 10 * max(L, M) */
    int32_t pre;           /* zero pre-pad of the prototype */
} XmResampleDesign;

XM_API int xm_resample_design(int in_rate, int out_rate, XmResampleDesign *d, float *H);

/* n_out = ceil(frames_in * L / M) for the reduced ratio (0 on bad rates). */
XM_API size_t xm_resample_out_frames(int in_rate, int out_rate, size_t frames_in);

/* ---- synthetic PCM in device memory (benchmarks / tests)
 * Clip c (c < n_clips) is written at dst + c*frames*channels samples with
 * clip id clip0 + c:  idx = (id << 32) | (frame*channels + ch),
 * z = splitmix64_mix(seed + idx * 0x9E3779B97F4A7C15),
 * F32: ((int)(z >> 40) - 2^23) * 2^-23  (uniform in [-1, 1), exact)
 * S16: (int16)(z >> 48).
 * dst must be device memory of `device` (host memory for XM_DEVICE_CPU);
 * stream may be NULL (synchronous). */
XM_API int xm_synth_pcm(void *dst, int sample_fmt, uint64_t seed, uint64_t clip0, int64_t n_clips,
                 int channels, int64_t frames, int device, void *hip_stream);

#ifdef __cplusplus
}
#endif
#endif /* XM_AUDIO_COMMON_H */
