// xm_device.h — device-side helpers shared by the gfx950 kernels.
// Arithmetic contract: include/xm_audio_common.h.  Every fp32 op here is a
// separately rounded IEEE op: the library is compiled with -ffp-contract=off
// and uses no fast-math, so hipcc never fuses a mul+add into an FMA.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "xm_gpu.h"

#define XM_DEV __device__ __forceinline__

// Per-output-frame fp32 gain (xm_audio_common.h "Gain ramp", F32).
XM_DEV float xm_gain_f32(const XmhGain &g, int64_t n)
{
    float v;
    if (g.len == 0) {
        v = n >= g.start ? g.g1 : g.g0;
    } else {
        int64_t k = n - g.start;
        k = k < 0 ? 0 : (k > g.len ? g.len : k);
        v = g.g0 + g.step * (float)(int32_t)k;
    }
    return (g.flags & XMH_GAIN_XFADE_OUT) ? 1.0f - v : v;
}

// Per-output-frame Q15 gain (xm_audio_common.h "Gain ramp", Q15).
XM_DEV int32_t xm_gain_q15(const XmhGain &g, int64_t n)
{
    int32_t v;
    if (g.len == 0) {
        v = n >= g.start ? g.q1 : g.q0;
    } else {
        int64_t k = n - g.start;
        k = k < 0 ? 0 : (k > g.len ? g.len : k);
        v = g.q0 + (int32_t)(((int64_t)(g.q1 - g.q0) * k) / g.len);  // C truncation
    }
    return (g.flags & XMH_GAIN_XFADE_OUT) ? 32768 - v : v;
}

// True when the gain is constant over output frames [n0, n1].
XM_DEV bool xm_gain_const(const XmhGain &g, int64_t n0, int64_t n1)
{
    if (g.len == 0) return n1 < g.start || n0 >= g.start;
    return n1 <= g.start || n0 >= g.start + g.len;
}

XM_DEV int16_t xm_sat16(int32_t v)
{
    return (int16_t)(v < -32768 ? -32768 : (v > 32767 ? 32767 : v));
}

// s16 track sample after fp32 resampling: lrintf (RNE) then saturate.
// rint, then v_cvt_i32_f32 (exact on the integer-valued float; it saturates
// past the int32 range and gives 0 for NaN), then one v_med3_i32: the same
// value as clamping in float first (the float clamp compiled to two compares
// and two selects per sample: 3 VALU instead of 6 per channel, round 6)
XM_DEV int32_t xm_round_sat16(float v)
{
    const float r = __builtin_rintf(v);      // v_rndne_f32: ties-to-even
    int32_t i;
    asm("v_cvt_i32_f32 %0, %1" : "=v"(i) : "v"(r));
    return i < -32768 ? -32768 : (i > 32767 ? 32767 : i);   // v_med3_i32
}

XM_DEV int32_t xm_q15_term(int32_t s, int32_t g)
{
    return (s * g + 16384) >> 15;            // s*g fits int32 for g <= 65535
}

XM_DEV const void *xm_track_ptr(const XmhMixJob &j, int b, int tr, int elem)
{
    if (j.in_ptrs) return j.in_ptrs[(int64_t)b * j.n_tracks + tr];
    return (const char *)j.in + ((int64_t)b * j.in_mix_stride + (int64_t)tr * j.in_track_stride) * elem;
}

XM_DEV void *xm_out_ptr(const XmhMixJob &j, int b, int elem)
{
    if (j.out_ptrs) return j.out_ptrs[b];
    return (char *)j.out + (int64_t)b * j.out_mix_stride * elem;
}
