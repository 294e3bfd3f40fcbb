// xm_resample_fast.hip — specialised gfx950 kernel for the headline path
// (48 kHz -> 44.1 kHz stereo fp32 resample + gain + ordered mix).
// Placeholder until the specialised kernel lands: declines every job so the
// generic LDS-staged kernel (xm_mix_generic.hip) runs.
#include "xm_device.h"

extern "C" int xmh_launch_mix_fast(const XmhMixJob *j, void *stream, int *n_launches)
{
    (void)j; (void)stream; (void)n_launches;
    return -1003;  // XM_ENOSYS: not handled here
}
