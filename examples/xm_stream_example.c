/*
 * xm_stream_example.c — a plain C caller of the streaming and timeline entry
 * points (INTEGRATION.md "Streams of blocks and timelines").
 *
 * 1. A 48 kHz stereo BGM + voice pair is fed to a 44.1 kHz mixer in ragged
 *    blocks (xm_audio_mixer_stream_push / _flush) and the concatenated output
 *    is compared, bit for bit, with one whole-signal process_batch call.
 * 2. The same biquad is streamed through xm_effects_process_stream and
 *    compared with xm_effects_process_batch.
 * 3. A timeline: BGM at 48 kHz from frame 0, a 16 kHz voice placed 0.5 s in,
 *    mixed to 44.1 kHz with a duck on the BGM (xm_audio_mixer_process_timeline).
 *
 * Exit status: 0 on success, 2 when no usable GPU is present (no CPU
 * fallback), 1 on any other error or mismatch.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "xm_audio_mixer.h"
#include "xm_effects.h"

#define N_IN 24000 /* 0.5 s @ 48 kHz */

static int fail(const char *what, int st)
{
    fprintf(stderr, "%s: %s (%d)\n", what, xm_strerror(st), st);
    return st == XM_EDEVICE ? 2 : 1;
}

static void tone(float *x, size_t frames, double hz, double rate, float amp)
{
    for (size_t i = 0; i < frames; ++i) {
        x[2 * i] = amp * (float)sin(6.283185307179586 * hz * (double)i / rate);
        x[2 * i + 1] = 0.5f * x[2 * i];
    }
}

int main(void)
{
    printf("%s, %d HIP device(s)\n", xm_version(), xm_device_count());
    int st = XM_OK;
    XmMixerConfig cfg = {0};
    cfg.in_rate = 48000;
    cfg.out_rate = 44100;
    cfg.channels = 2;
    cfg.sample_fmt = XM_FMT_F32;
    cfg.mem_kind = XM_MEM_HOST;
    cfg.n_devices = 1;   /* one GPU (0 would select the host CPU backend) */
    XmAudioMixer *mx = xm_audio_mixer_create_ex(&cfg, &st);
    if (!mx) return fail("xm_audio_mixer_create_ex", st);

    /* --- 1. streamed resample + mix == whole-signal call ------------------ */
    XmTrackDesc tr[2];
    memset(tr, 0, sizeof tr);
    tr[0].gain.gain0 = 0.8f; tr[0].gain.gain1 = 0.3f;          /* duck the BGM */
    tr[0].gain.ramp_start = 8000; tr[0].gain.ramp_len = 4410;
    tr[1].gain.gain0 = 1.0f; tr[1].gain.gain1 = 1.0f;
    if ((st = xm_audio_mixer_set_tracks(mx, tr, 2))) return fail("set_tracks", st);
    float *in = malloc(sizeof(float) * 2 * 2 * N_IN);          /* [track][frame][ch] */
    tone(in, N_IN, 220.0, 48000.0, 0.5f);
    tone(in + 2 * N_IN, N_IN, 1000.0, 48000.0, 0.4f);
    const size_t F = xm_audio_mixer_out_frames(mx, N_IN);
    float *whole = malloc(sizeof(float) * 2 * F), *streamed = malloc(sizeof(float) * 2 * F);
    const void *ins[2] = {in, in + 2 * N_IN};
    void *outs[1] = {whole};
    if ((st = xm_audio_mixer_process_batch(mx, ins, outs, 1, N_IN))) return fail("process_batch", st);

    /* the stream sees the tracks as one [track][frame][ch] block per push */
    static const size_t blocks[] = {1, 0, 37, 1000, 4096, 3, 8000};
    size_t pushed = 0, got = 0, n_out = 0;
    float *blk = malloc(sizeof(float) * 2 * 2 * N_IN);
    if ((st = xm_audio_mixer_stream_begin(mx, 1))) return fail("stream_begin", st);
    for (size_t k = 0; pushed < N_IN; ++k) {
        size_t n = k < sizeof blocks / sizeof blocks[0] ? blocks[k] : 5000;
        if (n > N_IN - pushed) n = N_IN - pushed;
        for (int t = 0; t < 2; ++t)
            memcpy(blk + 2 * n * t, in + 2 * (N_IN * t + pushed), sizeof(float) * 2 * n);
        const size_t want = xm_audio_mixer_stream_out_frames(mx, n, 0);
        st = xm_audio_mixer_stream_push(mx, blk, (ptrdiff_t)(2 * n), (ptrdiff_t)(4 * n), n, streamed + 2 * got,
                                        (ptrdiff_t)(2 * F), F - got, &n_out);
        if (st) return fail("stream_push", st);
        if (n_out != want) return fail("stream_push count", XM_EINVAL);
        got += n_out;
        pushed += n;
    }
    if ((st = xm_audio_mixer_stream_flush(mx, streamed + 2 * got, (ptrdiff_t)(2 * F), F - got, &n_out)))
        return fail("stream_flush", st);
    got += n_out;
    if (got != F || memcmp(whole, streamed, sizeof(float) * 2 * F) != 0) {
        fprintf(stderr, "streamed mix differs from the whole-signal mix (%zu of %zu frames)\n", got, F);
        return 1;
    }
    printf("stream mix: %zu frames, bit-identical to process_batch\n", got);

    /* --- 2. streamed effects == whole-signal effects ---------------------- */
    XmEffectsConfig ec = {44100, 2, XM_MEM_HOST, 0};
    XmEffects *fx = xm_effects_create_ex(&ec, &st);
    if (!fx) return fail("xm_effects_create_ex", st);
    if ((st = xm_effects_add_eq_band(fx, XM_EQ_PEAKING, 1000.0, 6.0, 1.0))) return fail("add_eq_band", st);
    static const float h[5] = {0.1f, 0.2f, 0.4f, 0.2f, 0.1f};
    if ((st = xm_effects_add_fir(fx, h, 5))) return fail("add_fir", st);
    float *fw = malloc(sizeof(float) * 2 * F), *fs = malloc(sizeof(float) * 2 * F);
    const float *fin[1] = {whole};
    float *fout[1] = {fw};
    if ((st = xm_effects_process_batch(fx, fin, fout, 1, F))) return fail("effects_process_batch", st);
    if ((st = xm_effects_stream_reset(fx, 1))) return fail("effects_stream_reset", st);
    for (size_t p = 0, k = 0; p < F; ++k) {
        size_t n = 1 + (k * 977) % 3001;
        if (n > F - p) n = F - p;
        const float *bi[1] = {whole + 2 * p};
        float *bo[1] = {fs + 2 * p};
        if ((st = xm_effects_process_stream(fx, bi, bo, 1, n))) return fail("effects_process_stream", st);
        p += n;
    }
    if (memcmp(fw, fs, sizeof(float) * 2 * F) != 0) {
        fprintf(stderr, "streamed effects differ from process_batch\n");
        return 1;
    }
    printf("stream effects: %zu frames, bit-identical to process_batch\n", F);

    /* --- 3. timeline: 48 kHz BGM + 16 kHz voice placed at 0.5 s ----------- */
    const size_t NV = 8000;                                   /* 0.5 s @ 16 kHz */
    float *voice = malloc(sizeof(float) * 2 * NV);
    tone(voice, NV, 300.0, 16000.0, 0.6f);
    tr[1].in_rate = 16000;
    if ((st = xm_audio_mixer_set_tracks(mx, tr, 2))) return fail("set_tracks (16 kHz voice)", st);
    const size_t FT = 44100;                                  /* 1 s of output */
    float *tl = malloc(sizeof(float) * 2 * FT);
    XmTrackPlacement pl[2] = {{0, N_IN}, {22050, (int64_t)NV}};
    const void *tin[2] = {in, voice};
    void *tout[1] = {tl};
    if ((st = xm_audio_mixer_process_timeline(mx, tin, pl, tout, 1, FT))) return fail("process_timeline", st);
    double e0 = 0, e1 = 0;
    for (size_t i = 0; i < 2 * 22050; ++i) e0 += (double)tl[i] * tl[i];
    for (size_t i = 2 * 22050; i < 2 * FT; ++i) e1 += (double)tl[i] * tl[i];
    printf("timeline: %zu frames, rms first half %.4f, second half %.4f\n", FT, sqrt(e0 / (2 * 22050)),
           sqrt(e1 / (2 * 22050)));
    if (!(e0 > 0 && e1 > 0)) return 1;

    xm_effects_freep(&fx);
    xm_audio_mixer_freep(&mx);
    free(in); free(whole); free(streamed); free(blk); free(fw); free(fs); free(voice); free(tl);
    return 0;
}
