/*
 * xm_mix_example.c — a plain C caller of the drop-in API.
 *
 * Mixes 2 mixes x 8 stereo fp32 tracks at 48 kHz down to 44.1 kHz with a BGM
 * duck, a crossfade pair and a fade-out, from HOST memory (the library stages
 * HBM itself), then runs a 5-band EQ chain with xm_effects_* on the result.
 *
 *   gcc -std=c11 -O2 -I include examples/xm_mix_example.c \
 *       -L xm-audio-utils_amd/lib -lxm_audio -Wl,-rpath,$PWD/xm-audio-utils_amd/lib -lm
 *
 * Exit status: 0 on success, 2 when no usable GPU is present (the library has
 * no CPU fallback and says so), 1 on any other error.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "xm_audio_mixer.h"
#include "xm_effects.h"

#define NT 8
#define NMIX 2
#define FRAMES_IN 48000 /* 1 s @ 48 kHz */
#define TWO_PI 6.283185307179586

static int fail(const char *what, int st)
{
    fprintf(stderr, "%s: %s (%d)\n", what, xm_strerror(st), st);
    return st == XM_EDEVICE ? 2 : 1;
}

int main(void)
{
    printf("%s, %d HIP device(s)\n", xm_version(), xm_device_count());

    XmMixerConfig cfg = {0};
    cfg.in_rate = 48000;
    cfg.out_rate = 44100;
    cfg.channels = 2;
    cfg.sample_fmt = XM_FMT_F32;
    cfg.mem_kind = XM_MEM_HOST;
    cfg.device = 0;
    cfg.n_devices = 1;   /* one GPU (0 would select the host CPU backend) */
    int st = 0;
    XmAudioMixer *mx = xm_audio_mixer_create_ex(&cfg, &st);
    if (!mx) return fail("xm_audio_mixer_create_ex", st);

    /* track 0: voice at unity; 1: BGM ducked 0.8 -> 0.3 over 0.25 s from 0.5 s;
     * 2/3: crossfade over 0.2 s at 0.3 s; 4..7: constant 0.1; 7 fades out */
    XmTrackDesc tr[NT];
    memset(tr, 0, sizeof tr);
    for (int i = 0; i < NT; ++i) {
        tr[i].gain.gain0 = tr[i].gain.gain1 = i == 0 ? 1.0f : 0.1f;
        tr[i].gain.gain0_q15 = tr[i].gain.gain1_q15 = 32768;
    }
    tr[1].gain.gain0 = 0.8f;
    tr[1].gain.gain1 = 0.3f;
    tr[1].gain.ramp_start = 22050;
    tr[1].gain.ramp_len = 11025;
    tr[7].gain.gain0 = 0.1f;
    tr[7].gain.gain1 = 0.0f;
    tr[7].gain.ramp_start = 33075;
    tr[7].gain.ramp_len = 11025;
    if ((st = xm_audio_mixer_set_tracks(mx, tr, NT))) return fail("set_tracks", st);
    if ((st = xm_audio_mixer_set_crossfade(mx, 2, 3, 13230, 8820))) return fail("set_crossfade", st);

    const size_t fout = xm_audio_mixer_out_frames(mx, FRAMES_IN);
    float *in = malloc(sizeof(float) * (size_t)NMIX * NT * FRAMES_IN * 2);
    float *out = malloc(sizeof(float) * (size_t)NMIX * fout * 2);
    if (!in || !out) return 1;
    const void *in_ptrs[NMIX * NT];
    void *out_ptrs[NMIX];
    for (int b = 0; b < NMIX; ++b) {
        out_ptrs[b] = out + (size_t)b * fout * 2;
        for (int t = 0; t < NT; ++t) {
            float *x = in + ((size_t)b * NT + t) * FRAMES_IN * 2;
            const double f = 110.0 * (t + 1) * (b + 1);
            for (int n = 0; n < FRAMES_IN; ++n) {
                x[2 * n] = (float)(0.5 * sin(TWO_PI * f * n / 48000.0));
                x[2 * n + 1] = (float)(0.5 * cos(TWO_PI * f * n / 48000.0));
            }
            in_ptrs[b * NT + t] = x;
        }
    }
    if ((st = xm_audio_mixer_process_batch(mx, in_ptrs, out_ptrs, NMIX, FRAMES_IN)))
        return fail("process_batch", st);
    XmMixerTiming tm;
    xm_audio_mixer_get_timing(mx, &tm);

    /* 5-band EQ on the two mixes (in place) */
    XmEffects *fx = xm_effects_create(44100, 2, 1);
    if (!fx) return fail("xm_effects_create", XM_EDEVICE);
    const int type[5] = {XM_EQ_LOWSHELF, XM_EQ_PEAKING, XM_EQ_PEAKING, XM_EQ_PEAKING, XM_EQ_HIGHSHELF};
    const double f0[5] = {80, 250, 1000, 4000, 12000}, gdb[5] = {3, -2, 1, 2, -1};
    const double q[5] = {1.0, 0.707, 0.707, 0.707, 1.0};   /* shelves: slope S */
    for (int i = 0; i < 5; ++i)
        if ((st = xm_effects_add_eq_band(fx, type[i], f0[i], gdb[i], q[i]))) return fail("add_eq_band", st);
    const float *fin[NMIX] = {out, out + fout * 2};
    float *fo[NMIX] = {out, out + fout * 2};
    if ((st = xm_effects_process_batch(fx, fin, fo, NMIX, fout))) return fail("effects_process", st);

    for (int b = 0; b < NMIX; ++b) {
        double e = 0;
        for (size_t i = 0; i < fout * 2; ++i) e += (double)out[b * fout * 2 + i] * out[b * fout * 2 + i];
        printf("mix %d: %zu frames @44.1k, rms %.4f\n", b, fout, sqrt(e / (fout * 2)));
    }
    printf("mixer: h2d %.3f ms, kernels %.3f ms (%d launches), d2h %.3f ms\n", tm.h2d_ms, tm.kernel_ms,
           tm.n_launches, tm.d2h_ms);
    xm_effects_freep(&fx);
    xm_audio_mixer_freep(&mx);
    free(in);
    free(out);
    return mx == NULL && fx == NULL ? 0 : 1;
}
