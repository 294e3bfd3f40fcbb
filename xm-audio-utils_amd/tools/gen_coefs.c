/*
 * gen_coefs.c — build-time generator for the fast 48k->44.1k kernel's
 * coefficient header.  Runs xm_resample_design(48000, 44100) (src/xm_design.c,
 * the scipy restatement) and writes, in output order within a super-period,
 *
 *     kH147[k][t] = H[((k + rm) * M) % L][t],  k < 147, t < 22
 *
 * as exact hex-float literals, so every v_mul_f32 in the kernel carries its
 * coefficient inline (no scalar loads).  Tap 22 of every phase must be an exact
 * zero (the 160-frame pre-pad); the generator refuses otherwise.
 *
 * and the 44.1k->48k tables (emit_up), the 44.1k->96k / 22.05k->48k ones
 * (emit_offsets "U2": L/M = 320/147), and the small-ratio pair tables
 * (emit_ratio: 3/2, 2/3, 1/2, 2/1, 3/1).
 *
 * usage: gen_coefs <out.h>
 */
#include <stdio.h>
#include <stdlib.h>

#include "xm_audio_common.h"

/* 44.1k -> 48k (L/M = 160/147, T = 21): tap 0 is an exact zero in 142 of the
 * 160 phases and tap 20 in 17 (the prototype's ends fall outside the phase),
 * so output k uses the contiguous taps kOffU[k] .. kOffU[k] + n_k - 1, with
 * n_k = 20 except for one output (21).  The packed table pairs outputs
 * (2i, 2i+1) by their *used* taps: kHpU[i][2e + j] = H[ph(2i+j)][kOffU[2i+j]
 * + e], and a pair runs max(n_2i, n_2i+1) taps (kPtU[i]); the shorter output
 * gets +0 coefficients past its end (acc + x*0 == acc up to the sign of zero,
 * which the kernel's final + 0 fixes; finite inputs), and the leading zero
 * taps are dropped like the 147/160 kernel's tap 22. */
/* The same per-output used-tap runs for any L (even) / M with T = 21 (emit_up
 * for 160/147; 320/147 = 44.1k -> 96k and 22.05k -> 48k as "U2"): emits
 * XM_FAST_RM_<sfx>, kOff<sfx>[L], kPt<sfx>[L / 2] and XM_KHP<sfx>_INIT[L / 2 +
 * 1][42]. */
static int emit_offsets_t(FILE *f, const char *sfx, int in_rate, int out_rate, int Lx, int Mx, int Tx, int ptmin, int ptmax);
static int emit_offsets(FILE *f, const char *sfx, int in_rate, int out_rate, int Lx, int Mx)
{
    return emit_offsets_t(f, sfx, in_rate, out_rate, Lx, Mx, 21, 17, 21);
}

/* any T: also kNum<sfx>[L] (used taps of each output) */
static int emit_offsets_t(FILE *f, const char *sfx, int in_rate, int out_rate, int Lx, int Mx, int Tx, int ptmin, int ptmax)
{
    XmResampleDesign d;
    const int NP = (Lx + 1) / 2;   /* pairs; an odd L leaves the last output unpaired (+0 partner) */
    float *H = calloc((size_t)Lx * Tx, sizeof(float));
    int *off = calloc((size_t)Lx, sizeof(int)), *n = calloc((size_t)Lx, sizeof(int)), *pt = calloc((size_t)NP, sizeof(int));
    int rc = 1;
    if (!H || !off || !n || !pt || xm_resample_design(in_rate, out_rate, &d, NULL) || d.L != Lx || d.M != Mx ||
        d.T != Tx || xm_resample_design(in_rate, out_rate, &d, H)) {
        fprintf(stderr, "gen_coefs: unexpected %d -> %d design\n", in_rate, out_rate);
        goto out;
    }
    for (int k = 0; k < Lx; ++k) {
        const int ph = (int)(((long)(k + d.rm) * Mx) % Lx);
        int lo = -1, hi = -1;
        for (int t = 0; t < Tx; ++t)
            if (H[ph * Tx + t] != 0.0f) {
                if (lo < 0) lo = t;
                hi = t;
            }
        if (lo < 0) goto out;
        off[k] = lo;   /* interior zero taps, if any, stay in the chain */
        n[k] = hi - lo + 1;
    }
    for (int i = 0; i < NP; ++i) {
        const int n1 = 2 * i + 1 < Lx ? n[2 * i + 1] : 0;
        pt[i] = n[2 * i] > n1 ? n[2 * i] : n1;
        if (pt[i] < ptmin || pt[i] > ptmax) {
            fprintf(stderr, "gen_coefs: %s pair %d runs %d taps\n", sfx, i, pt[i]);
            goto out;
        }
    }
    fprintf(f, "// %d -> %d (xm_resample_design(%d, %d)): L = %d, M = %d, T = %d\n", in_rate, out_rate, in_rate,
            out_rate, Lx, Mx, Tx);
    fprintf(f, "#define XM_FAST_RM_%s %d\n", sfx, d.rm);
    fprintf(f, "static constexpr int kOff%s[%d] = {", sfx, Lx);
    for (int k = 0; k < Lx; ++k) fprintf(f, "%s%d", k ? ", " : "", off[k]);
    fprintf(f, "};\nstatic constexpr int kNum%s[%d] = {", sfx, Lx);
    for (int k = 0; k < Lx; ++k) fprintf(f, "%s%d", k ? ", " : "", n[k]);
    fprintf(f, "};\nstatic constexpr int kPt%s[%d] = {", sfx, NP);
    for (int i = 0; i < NP; ++i) fprintf(f, "%s%d", i ? ", " : "", pt[i]);
    fprintf(f, "};\n#define XM_KHP%s_INIT { \\\n", sfx);
    for (int i = 0; i <= NP; ++i) {   /* + 1 zero row: prefetch past the end stays in bounds */
        fprintf(f, "  {");
        for (int e = 0; e < ptmax; ++e)
            for (int j = 0; j < 2; ++j) {
                const int k = 2 * i + j;
                const float v = k < Lx && e < n[k] ? H[(int)(((long)(k + d.rm) * Mx) % Lx) * Tx + off[k] + e] : 0.0f;
                fprintf(f, "%s%af", e || j ? ", " : "", (double)v);
            }
        fprintf(f, "}, \\\n");
    }
    fprintf(f, "}\n");
    rc = 0;
out:
    free(H);
    free(off);
    free(n);
    free(pt);
    return rc;
}

static int emit_up(FILE *f) { return emit_offsets(f, "U", 44100, 48000, 160, 147); }

/* The small-L/M ratios of the fused kernel (RatioBase<RID> in
 * csrc/xm_resample_fast.hip): every output runs all T taps, and the phase of
 * output k, ((k + rm) * M) % L, repeats every L outputs, so the pair rows
 * (outputs 2i, 2i+1) repeat every PR = L / gcd(L, 2) pairs.  Emits
 *     XM_R<name>_RM, XM_R<name>_T, XM_R<name>_PR and
 *     XM_KHP<name>_INIT[PR + 1][2T]: row i = (h_2i[t], h_2i+1[t]) for t < T,
 * plus one zero row (the last coefficient group of a row reads up to 16
 * floats past its start).  The design depends on L and M only. */
static int emit_ratio(FILE *f, const char *name, int L, int M)
{
    XmResampleDesign d;
    if (xm_resample_design(M, L, &d, NULL) || d.L != L || d.M != M) return 1;
    float *H = calloc((size_t)(L * d.T), sizeof(float));
    if (!H || xm_resample_design(M, L, &d, H)) {
        free(H);
        return 1;
    }
    const int PR = L % 2 ? L : L / 2;
    fprintf(f, "// %d/%d (xm_resample_design(%d, %d)): T = %d, rm = %d, pair rows repeat every %d\n", L, M, M, L, d.T,
            d.rm, PR);
    fprintf(f, "#define XM_R%s_RM %d\n#define XM_R%s_T %d\n#define XM_R%s_PR %d\n", name, d.rm, name, d.T, name, PR);
    fprintf(f, "#define XM_KHP%s_INIT { \\\n", name);
    for (int i = 0; i <= PR; ++i) {
        fprintf(f, "  {");
        for (int t = 0; t < d.T; ++t)
            for (int j = 0; j < 2; ++j) {
                const int k = 2 * i + j;
                const float v = i < PR ? H[(((k + d.rm) * M) % L) * d.T + t] : 0.0f;
                fprintf(f, "%s%af", t || j ? ", " : "", (double)v);
            }
        fprintf(f, "}, \\\n");
    }
    fprintf(f, "}\n");
    free(H);
    return 0;
}

int main(int argc, char **argv)
{
    if (argc != 2) {
        fprintf(stderr, "usage: %s out.h\n", argv[0]);
        return 2;
    }
    XmResampleDesign d;
    float H[147 * 23];
    if (xm_resample_design(48000, 44100, &d, NULL) || d.L != 147 || d.M != 160 || d.T != 23 ||
        xm_resample_design(48000, 44100, &d, H)) {
        fprintf(stderr, "gen_coefs: unexpected 48k->44.1k design\n");
        return 1;
    }
    for (int ph = 0; ph < 147; ++ph)
        if (H[ph * 23 + 22] != 0.0f) {
            fprintf(stderr, "gen_coefs: tap 22 of phase %d is not zero\n", ph);
            return 1;
        }
    FILE *f = fopen(argv[1], "w");
    if (!f) {
        perror(argv[1]);
        return 1;
    }
    fprintf(f, "// generated by tools/gen_coefs.c from xm_resample_design(48000, 44100); do not edit\n");
    fprintf(f, "// kH147[k][t] = H[((k + %d) * 160) %% 147][t]: output k of a super-period, tap t\n", d.rm);
    fprintf(f, "#pragma once\n#define XM_FAST_RM %d\n", d.rm);
    fprintf(f, "static constexpr float kH147[147][22] = {\n");
    for (int k = 0; k < 147; ++k) {
        const int ph = ((k + d.rm) * 160) % 147;
        fprintf(f, "  {");
        for (int t = 0; t < 22; ++t) fprintf(f, "%s%af", t ? ", " : "", (double)H[ph * 23 + t]);
        fprintf(f, "},\n");
    }
    fprintf(f, "};\n");
    /* pair-interleaved form for the packed-math taps: kHp147[i][2t + j] =
     * H[ph(2i + j)][t], the unpaired last output (k = 146) gets a 0 partner */
    fprintf(f, "#define XM_KHP147_INIT { \\\n");
    for (int i = 0; i < 74; ++i) {
        fprintf(f, "  {");
        for (int t = 0; t < 22; ++t)
            for (int j = 0; j < 2; ++j) {
                const int k = 2 * i + j;
                const float v = k < 147 ? H[(((k + d.rm) * 160) % 147) * 23 + t] : 0.0f;
                fprintf(f, "%s%af", t || j ? ", " : "", (double)v);
            }
        fprintf(f, "}, \\\n");
    }
    fprintf(f, "}\n");
    return emit_up(f) || emit_offsets(f, "U2", 44100, 96000, 320, 147) ||
                   emit_offsets_t(f, "D2", 96000, 44100, 147, 320, 46, 43, 44) || emit_ratio(f, "32", 3, 2) || emit_ratio(f, "23", 2, 3) || emit_ratio(f, "12", 1, 2) ||
                   emit_ratio(f, "21", 2, 1) || emit_ratio(f, "31", 3, 1) || fclose(f)
               ? 1
               : 0;
}
