/*
 * xm_oracle.h — C restatement of the PCM hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Used by tests/ (parity at scale), __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg — never by the product library, which has no CPU path.
 * Same arithmetic as oracle/np_oracle.py (pinned bit-exact to scipy 1.15.3
 * golden vectors in tests/golden/), compiled with -ffp-contract=off so every
 * fp32 mul and add is rounded separately.
 * "Parity vs the reference": the reference has no code (README.md:1); parity
 * is pinned to scipy, the third-party algorithm BASELINE.json:5 names.
 */
#ifndef XM_ORACLE_H
#define XM_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#include "xm_audio_common.h"

#ifdef __cplusplus
extern "C" {
#endif

void xo_gen_f32(uint64_t seed, uint64_t clip, int channels, size_t frames, float *out);
void xo_gen_s16(uint64_t seed, uint64_t clip, int channels, size_t frames, int16_t *out);

size_t xo_resample_out_frames(size_t n, int L, int M);
/* x: N frames x C channels interleaved -> y: ceil(N*L/M) frames x C */
void xo_resample_f32(const float *H, int L, int M, int T, int rm,
                     const float *x, size_t N, int C, float *y);
void xo_resample_s16(const float *H, int L, int M, int T, int rm,
                     const int16_t *x, size_t N, int C, int16_t *y);

float   xo_gain_f32(const XmGainRamp *r, int64_t n);
int32_t xo_gain_q15(const XmGainRamp *r, int64_t n);

/* r[tr]: F frames x C, already at output rate */
void xo_mix_f32(const float *const *r, const XmGainRamp *g, int ntr, size_t F, int C, float *out);
void xo_mix_s16(const int16_t *const *s, const XmGainRamp *g, int ntr, size_t F, int C, int16_t *out);

/* resample every track (N frames in) then mix; scratch-free per call */
void xo_resample_mix_f32(const float *H, int L, int M, int T, int rm,
                         const float *const *x, const XmGainRamp *g, int ntr,
                         size_t N, int C, float *out);
void xo_resample_mix_s16(const float *H, int L, int M, int T, int rm,
                         const int16_t *const *x, const XmGainRamp *g, int ntr,
                         size_t N, int C, int16_t *out);

/* sos: nsec x 6 (b0 b1 b2 a0 a1 a2), a0 == 1 */
void xo_biquad_f32(const float *sos, int nsec, const float *x, size_t N, int C, float *y);
void xo_fir_f32(const float *h, int K, const float *x, size_t N, int C, float *y);

/* CPU-baseline driver: nmix mixes of ntr tracks, each track a strided slice of
 * `in` (track tr of mix b at in + (b*ntr+tr)*N*C), out at out + b*Fout*C.
 * Uses `threads` OpenMP threads over mixes (1 = scalar port).  Returns the
 * number of threads actually used. */
int xo_batch_resample_mix_f32(const float *H, int L, int M, int T, int rm,
                              const float *in, const XmGainRamp *g, int ntr,
                              size_t nmix, size_t N, int C, float *out, int threads);
int xo_batch_mix_s16(const int16_t *in, const XmGainRamp *g, int ntr, size_t nmix,
                     size_t F, int C, int16_t *out, int threads);

#ifdef __cplusplus
}
#endif
#endif
