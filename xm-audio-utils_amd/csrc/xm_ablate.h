/*
 * xm_ablate.h — the fused kernel's ablation switches (csrc/xm_resample_fast.hip).
 *
 * Diagnostic builds only: tools/dev/ab_part.sh rebuilds the kernel's parts
 * with -DXM_AB_<NAME> into a copy of the library, to time the kernel's halves
 * apart.  The product build defines none of them, so every
 * constant below is false / its default and each `if constexpr` on them
 * compiles away; every one but XM_AB_PRIO and XM_AB_DMAPOL breaks the result.
 *   XM_AB_NOWAIT  copy_seg issues no vmcnt wait (the DMA's latency hidden for free)
 *   XM_AB_NODMA   no LDS-DMA instruction (copies read whatever the slot holds)
 *   XM_AB_NOTAPS  no packed taps and no coefficient loads (the memory half alone)
 *   XM_AB_NOBAR   no s_barrier per super-period
 *   XM_AB_NOSTORE every output store dropped (out of range: no HBM write)
 *   XM_AB_NOEXCH  no exchange through LDS (track sums of constants)
 *   XM_AB_NOCOPY  no slot -> register copy (f32 interleaved kernels)
 *   XM_AB_PPP=n   DMA parts per output pair (a segment's DMA over 8 / n pairs)
 *   XM_AB_ROW0    every coefficient group read from table row 0 (no scalar-cache misses)
 *   XM_AB_PRIO=n  s_setprio 1 for waves 4-7 (n = 1), 0-3 (2) or the odd waves (3)
 *   XM_AB_DMAPOL=n the input DMA's cache policy for every instantiation: 0 nt, 1 sc1, 2 default
 *                 (the product: sc1 where segments straddle lines, nt elsewhere; this
 *                 one keeps the result)
 *   XM_AB_DSFAUX=n the cache-policy bits of the DSF / DS grouped mono stores; XM_AB_MONOAUX=n
 *                 the other mono stores; XM_AB_SPLITAUX=n split mode's whole-segment (SEG) stores;
 *                 XM_AB_PSPLITAUX=n split mode's plain stores; XM_AB_MIXAUX=n the interleaved f32
 *                 mixes' round stores (each keeps the result)
 *   XM_AB_SEGALL  the segment stores (SEG) for the 2- and 4-track split layouts too (keeps the result)
 *   XM_AB_NOMISSEG no segment stores for the 160/147 and 320/147 1-track rows (keeps the result)
 */
#ifndef XM_ABLATE_H
#define XM_ABLATE_H

namespace xm_ab {
#ifdef XM_AB_NOWAIT
constexpr bool kNoWait = true;
#else
constexpr bool kNoWait = false;
#endif
#ifdef XM_AB_NODMA
constexpr bool kNoDma = true;
#else
constexpr bool kNoDma = false;
#endif
#ifdef XM_AB_NOTAPS
constexpr bool kNoTaps = true;
#else
constexpr bool kNoTaps = false;
#endif
#ifdef XM_AB_NOBAR
constexpr bool kNoBar = true;
#else
constexpr bool kNoBar = false;
#endif
#ifdef XM_AB_NOSTORE
constexpr bool kNoStore = true;
#else
constexpr bool kNoStore = false;
#endif
#ifdef XM_AB_NOEXCH
constexpr bool kNoExch = true;
#else
constexpr bool kNoExch = false;
#endif
#ifdef XM_AB_NOCOPY
constexpr bool kNoCopy = true;
#else
constexpr bool kNoCopy = false;
#endif
#ifdef XM_AB_ROW0
constexpr bool kRow0 = true;
#else
constexpr bool kRow0 = false;
#endif
#ifdef XM_AB_PPP
constexpr int kPPP = XM_AB_PPP;
#else
constexpr int kPPP = 1;
#endif
#ifdef XM_AB_PRIO
constexpr int kPrio = XM_AB_PRIO;
#else
constexpr int kPrio = 0;
#endif
#ifdef XM_AB_DMAPOL
constexpr int kDmaPol = XM_AB_DMAPOL;
#else
constexpr int kDmaPol = -1;
#endif
#ifdef XM_AB_DSFAUX
constexpr int kDsfAux = XM_AB_DSFAUX;
#else
constexpr int kDsfAux = -1;
#endif
#ifdef XM_AB_MONOAUX
constexpr int kMonoAux = XM_AB_MONOAUX;
#else
constexpr int kMonoAux = -1;
#endif
#ifdef XM_AB_SPLITAUX
constexpr int kSplitAux = XM_AB_SPLITAUX;
#else
constexpr int kSplitAux = -1;
#endif
#ifdef XM_AB_SEGALL
constexpr bool kSegAll = true;
#else
constexpr bool kSegAll = false;
#endif
#ifdef XM_AB_NOMISSEG
constexpr bool kNoMisSeg = true;
#else
constexpr bool kNoMisSeg = false;
#endif
#ifdef XM_AB_MIXAUX
constexpr int kMixAux = XM_AB_MIXAUX;
#else
constexpr int kMixAux = -1;
#endif
#ifdef XM_AB_PSPLITAUX
constexpr int kPSplitAux = XM_AB_PSPLITAUX;
#else
constexpr int kPSplitAux = -1;
#endif
}  // namespace xm_ab

#endif /* XM_ABLATE_H */
