/*
 * xm_config1_cpu.c — BASELINE.json config 1 through the drop-in C API on the
 * host CPU backend, no GPU: one mono 10 s clip of synthetic s16 PCM at
 * 44.1 kHz resampled to 48 kHz ("xm_audio_mixer_process_batch
 * -> L2 sees devices=0 -> L0-cpu").
 *
 *   gcc -std=c11 -O2 -Iinclude examples/xm_config1_cpu.c -Lxm-audio-utils_amd/lib -lxm_audio -o cfg1
 *   ./cfg1 [out.raw]      (writes the 480000 s16 samples when a path is given)
 *
 * The clip is xm_synth_pcm's clip 0 with the bench seed, the input of the
 * committed config-1 digest (tests/golden/MANIFEST.json config1_sha256).
 */
#define _POSIX_C_SOURCE 199309L
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "xm_audio_mixer.h"

static int fail(const char *what, int st)
{
    fprintf(stderr, "%s: %s (%d)\n", what, xm_strerror(st), st);
    return 2;
}

int main(int argc, char **argv)
{
    enum { N_IN = 441000 };
    XmMixerConfig cfg = {0};
    cfg.in_rate = 44100;
    cfg.out_rate = 48000;
    cfg.channels = 1;
    cfg.sample_fmt = XM_FMT_S16;
    cfg.mem_kind = XM_MEM_HOST;
    cfg.n_devices = 0;   /* the host CPU backend (XM_DEVICE_CPU) */
    int st = 0;
    XmAudioMixer *mx = xm_audio_mixer_create_ex(&cfg, &st);
    if (!mx) return fail("xm_audio_mixer_create_ex", st);
    const size_t F = xm_audio_mixer_out_frames(mx, N_IN);
    int16_t *in = malloc(sizeof(int16_t) * N_IN), *out = malloc(sizeof(int16_t) * F);
    if (!in || !out) return fail("malloc", XM_ENOMEM);
    if ((st = xm_synth_pcm(in, XM_FMT_S16, 0x584D4155u, 0, 1, 1, N_IN, XM_DEVICE_CPU, NULL)))
        return fail("xm_synth_pcm", st);
    const void *ins[1] = {in};
    void *outs[1] = {out};
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    if ((st = xm_audio_mixer_process_batch(mx, ins, outs, 1, N_IN))) return fail("process_batch", st);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    const double s = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    uint64_t h = 1469598103934665603ull;   /* FNV-1a of the output bytes, for a quick look */
    for (size_t i = 0; i < F; ++i)
        for (int b = 0; b < 2; ++b) h = (h ^ (uint8_t)((uint16_t)out[i] >> (8 * b))) * 1099511628211ull;
    printf("config 1 (cpu backend): %zu -> %zu frames, %.3f ms, %.1f Msamples/s, fnv1a %016llx\n", (size_t)N_IN, F,
           s * 1e3, N_IN / s / 1e6, (unsigned long long)h);
    if (argc > 1) {
        FILE *f = fopen(argv[1], "wb");
        if (!f || fwrite(out, sizeof(int16_t), F, f) != F) return fail("write", XM_EINVAL);
        fclose(f);
    }
    xm_audio_mixer_freep(&mx);
    free(in);
    free(out);
    return mx == NULL ? 0 : 1;
}
