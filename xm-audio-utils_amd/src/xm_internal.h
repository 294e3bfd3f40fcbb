/*
 * xm_internal.h — host-side (C) internals shared by the API translation units.
 */
#ifndef XM_INTERNAL_H
#define XM_INTERNAL_H

#include "xm_audio_common.h"
#include "xm_audio_mixer.h"
#include "xm_effects.h"
#include "../csrc/xm_shim.h"

#define XM_MAX_TRACKS 64
#define XM_MAX_SOS 15   /* one wave per section + a loader wave <= 1024 threads (csrc/xm_fx.hip) */
#define XM_MAX_FIR 4096
#define XM_MAX_EFFECTS 32

/* Cached device resample table for one reduced ratio. */
typedef struct XmTable {
    XmResampleDesign d;
    float *H_dev;          /* L*T floats on the handle's device */
    int fast;              /* 1: the baked 147/160 kernel computes exactly this table */
} XmTable;

int  xm_table_build(XmTable *t, int in_rate, int out_rate);
void xm_table_free(XmTable *t);

/* Convert a public XmGainRamp to the device descriptor (validates ranges). */
int xm_gain_to_dev(const XmGainRamp *g, XmhGain *d);

/* Effects chain internals (used by the mixer for per-track chains). */
typedef struct XmFxStage {
    int kind;              /* 1 = biquad cascade, 2 = FIR */
    int n;                 /* sections or taps */
    float *coef_dev;       /* n*6 (biquad) or n (FIR) floats on device */
} XmFxStage;

int xm_effects_stages(const XmEffects *e, const XmFxStage **stages, int *n_stages);
int xm_effects_device(const XmEffects *e);

#endif
