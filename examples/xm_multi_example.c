/*
 * xm_multi_example.c — the multi-device form of the drop-in API from plain C
 * (SURVEY.md §8(b) n_devices; INTEGRATION.md "Multi-device handles").
 *
 *  1. A mixer over every visible GPU (XmMixerConfig.n_devices) resamples and
 *     mixes a batch from host memory: the library cuts the batch into one
 *     block of mixes per device, runs each block on its own worker thread and
 *     joins them.  The result is compared, bit for bit, with a one-device
 *     handle.  With a single GPU the device list [0, 0] stands in (two
 *     sub-handles on one device).
 *  2. Config 5: 64 s16 tracks per mix spread over the devices (device d holds
 *     tracks [d*64/n, (d+1)*64/n)), mixed by xm_audio_mixer_mix_spanning_s16
 *     (partials, one RCCL reduce-scatter, saturating finish), compared with a
 *     one-device 64-track mix.  The per-device buffers are the caller's: this
 *     example allocates them with the HIP runtime, so it links libamdhip64.
 *
 *   gcc -std=c11 -O2 -I include -I /opt/rocm/include -D__HIP_PLATFORM_AMD__ \
 *       examples/xm_multi_example.c -L xm-audio-utils_amd/lib -lxm_audio \
 *       -L /opt/rocm/lib -lamdhip64 -Wl,-rpath,$PWD/xm-audio-utils_amd/lib -lm
 *
 * Exit status: 0 on success, 2 when no usable GPU is present, 1 otherwise.
 */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "xm_audio_mixer.h"

#define NT 8
#define NMIX 5
#define FRAMES 24000
#define NT5 64
#define NMIX5 4
#define FRAMES5 9600

static int fail(const char *what, int st)
{
    fprintf(stderr, "%s: %s (%d)\n", what, xm_strerror(st), st);
    return st == XM_EDEVICE ? 2 : 1;
}

static unsigned lcg(unsigned *s) { return *s = *s * 1664525u + 1013904223u; }

int main(void)
{
    const int ndev = xm_device_count();
    printf("%s, %d HIP device(s)\n", xm_version(), ndev);
    if (ndev < 1) return fail("xm_device_count", XM_EDEVICE);
    int devs[16], n = ndev > 16 ? 16 : ndev;
    for (int d = 0; d < n; ++d) devs[d] = d;
    if (n == 1) devs[n++] = 0;   /* one GPU: two blocks on it */

    /* ---- 1. independent mixes, sharded over the devices --------------------- */
    XmMixerConfig cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.in_rate = 48000;
    cfg.out_rate = 44100;
    cfg.channels = 2;
    cfg.sample_fmt = XM_FMT_F32;
    cfg.mem_kind = XM_MEM_HOST;
    cfg.n_devices = 1;   /* one GPU (0 would select the host CPU backend) */
    int st = 0;
    XmAudioMixer *one = xm_audio_mixer_create_ex(&cfg, &st);
    if (!one) return fail("xm_audio_mixer_create_ex", st);
    XmAudioMixer *multi = xm_audio_mixer_create_multi(&cfg, devs, n, &st);
    if (!multi) return fail("xm_audio_mixer_create_multi", st);
    XmTrackDesc tr[NT];
    memset(tr, 0, sizeof tr);
    for (int t = 0; t < NT; ++t) {
        tr[t].gain.gain0 = 0.25f + 0.05f * (float)t;
        tr[t].gain.gain1 = 0.6f;
        tr[t].gain.ramp_start = 1000 * t;
        tr[t].gain.ramp_len = 4410;
    }
    if ((st = xm_audio_mixer_set_tracks(one, tr, NT)) || (st = xm_audio_mixer_set_tracks(multi, tr, NT)))
        return fail("set_tracks", st);
    if ((st = xm_audio_mixer_set_crossfade(multi, 6, 7, 5000, 8820)) ||
        (st = xm_audio_mixer_set_crossfade(one, 6, 7, 5000, 8820)))
        return fail("set_crossfade", st);
    const size_t fo = xm_audio_mixer_out_frames(one, FRAMES);
    float *x = malloc(sizeof(float) * NMIX * NT * FRAMES * 2);
    float *y1 = malloc(sizeof(float) * NMIX * fo * 2), *y2 = malloc(sizeof(float) * NMIX * fo * 2);
    if (!x || !y1 || !y2) return fail("malloc", XM_ENOMEM);
    unsigned seed = 12345u;
    for (size_t i = 0; i < (size_t)NMIX * NT * FRAMES * 2; ++i)
        x[i] = (float)((int)(lcg(&seed) >> 9) - (1 << 22)) * 0x1p-22f * 0.5f;
    const ptrdiff_t ts = FRAMES * 2, ms = NT * FRAMES * 2, os = (ptrdiff_t)fo * 2;
    if ((st = xm_audio_mixer_process_strided(one, x, ts, ms, y1, os, NMIX, FRAMES)))
        return fail("process_strided (one device)", st);
    if ((st = xm_audio_mixer_process_strided(multi, x, ts, ms, y2, os, NMIX, FRAMES)))
        return fail("process_strided (multi)", st);
    XmMixerTiming tm;
    xm_audio_mixer_get_timing(multi, &tm);
    if (memcmp(y1, y2, sizeof(float) * NMIX * fo * 2)) {
        fprintf(stderr, "multi-device mix differs from the one-device mix\n");
        return 1;
    }
    printf("sharded: %d mixes over %d devices, %d launches, bit-identical to one device\n", NMIX,
           xm_audio_mixer_n_devices(multi), tm.n_launches);
    xm_audio_mixer_freep(&multi);
    xm_audio_mixer_freep(&one);

    /* ---- 2. config 5: tracks spanning the devices ---------------------------- */
    int n5 = n;
    while (NT5 % n5 || NMIX5 % n5) --n5;   /* tracks and mixes split evenly */
    cfg.out_rate = 48000;
    cfg.sample_fmt = XM_FMT_S16;
    XmAudioMixer *ref = xm_audio_mixer_create_ex(&cfg, &st);
    if (!ref) return fail("create (reference)", st);
    cfg.mem_kind = XM_MEM_DEVICE;
    XmAudioMixer *span = xm_audio_mixer_create_multi(&cfg, devs, n5, &st);
    if (!span) return fail("create_multi (config 5)", st);
    XmTrackDesc t64[NT5];
    memset(t64, 0, sizeof t64);
    for (int t = 0; t < NT5; ++t) {
        t64[t].gain.gain0_q15 = 4096 + 512 * (t % 8);
        t64[t].gain.gain1_q15 = 40000 - 300 * t;
        t64[t].gain.ramp_start = 100 * t;
        t64[t].gain.ramp_len = 4800;
    }
    if ((st = xm_audio_mixer_set_tracks(ref, t64, NT5)) || (st = xm_audio_mixer_set_tracks(span, t64, NT5)))
        return fail("set_tracks (64)", st);
    const size_t per_mix = (size_t)NT5 * FRAMES5 * 2;
    int16_t *s = malloc(sizeof(int16_t) * NMIX5 * per_mix);
    int16_t *r = malloc(sizeof(int16_t) * NMIX5 * FRAMES5 * 2), *g = malloc(sizeof(int16_t) * NMIX5 * FRAMES5 * 2);
    if (!s || !r || !g) return fail("malloc", XM_ENOMEM);
    for (size_t i = 0; i < NMIX5 * per_mix; ++i) s[i] = (int16_t)(lcg(&seed) >> 16);
    if ((st = xm_audio_mixer_process_strided(ref, s, FRAMES5 * 2, (ptrdiff_t)per_mix, r, FRAMES5 * 2, NMIX5, FRAMES5)))
        return fail("process_strided (64 tracks)", st);
    /* device d: its tracks of every mix (contiguous [mix][track][frame][ch]) and its owned mixes */
    const int per = NT5 / n5, own = NMIX5 / n5;
    void *din[16], *dout[16];
    const size_t in_bytes = sizeof(int16_t) * NMIX5 * (size_t)per * FRAMES5 * 2;
    const size_t out_bytes = sizeof(int16_t) * own * FRAMES5 * 2;
    for (int d = 0; d < n5; ++d) {
        if (hipSetDevice(devs[d]) != hipSuccess || hipMalloc(&din[d], in_bytes) != hipSuccess ||
            hipMalloc(&dout[d], out_bytes) != hipSuccess)
            return fail("hipMalloc", XM_EDEVICE);
        for (int b = 0; b < NMIX5; ++b)
            if (hipMemcpy((char *)din[d] + (size_t)b * per * FRAMES5 * 2 * sizeof(int16_t),
                          s + b * per_mix + (size_t)d * per * FRAMES5 * 2, sizeof(int16_t) * per * FRAMES5 * 2,
                          hipMemcpyHostToDevice) != hipSuccess)
                return fail("hipMemcpy", XM_EDEVICE);
    }
    if ((st = xm_audio_mixer_mix_spanning_s16(span, (const void *const *)din, FRAMES5 * 2,
                                              (ptrdiff_t)per * FRAMES5 * 2, dout, FRAMES5 * 2, NMIX5, FRAMES5)))
        return fail("mix_spanning_s16", st);
    for (int d = 0; d < n5; ++d) {
        hipSetDevice(devs[d]);
        if (hipMemcpy(g + (size_t)d * own * FRAMES5 * 2, dout[d], out_bytes, hipMemcpyDeviceToHost) != hipSuccess)
            return fail("hipMemcpy", XM_EDEVICE);
        hipFree(din[d]);
        hipFree(dout[d]);
    }
    if (memcmp(r, g, sizeof(int16_t) * NMIX5 * FRAMES5 * 2)) {
        fprintf(stderr, "config-5 spanning mix differs from the one-device 64-track mix\n");
        return 1;
    }
    printf("config 5: %d mixes x %d tracks over %d devices, bit-identical to one device\n", NMIX5, NT5, n5);
    xm_audio_mixer_freep(&span);
    xm_audio_mixer_freep(&ref);
    free(x); free(y1); free(y2); free(s); free(r); free(g);
    return 0;
}
