// pulse_front.h — the audio pulse detector's per-sample front end, shared by the SSB kernels (ssb.hip runs it
// on each PCM sample it produces) and the standalone audio front-end kernel (pulse.hip).
//
// AudioPulseDetector::process(pcm) (src/ssb/audio_pulse_detector.cpp:92-110): x = pcm * (1/32767), the
// band-pass chain applyChain(bandSOS_) = HP(fMin) then LP(fMax) in direct form II transposed (:57-65),
// frameAcc_ += y^2, and every frameSamples_ samples the RMS through applyChain(lowSOS_) (:115) becomes one
// energy value for the detector.  Float expressions in the reference's order; callers compile with FP
// contraction off.
#pragma once

#include <hip/hip_runtime.h>

#include "sdrg_types.h"

namespace sdrg {

struct FrontState {
    float hz1, hz2, lz1, lz2, ez1, ez2, acc;
    int count;
};

__device__ __forceinline__ FrontState front_load(const PulseStreamState *g) {
    FrontState f;
    f.hz1 = g->band_z[0];
    f.hz2 = g->band_z[1];
    f.lz1 = g->band_z[2];
    f.lz2 = g->band_z[3];
    f.ez1 = g->low_z[0];
    f.ez2 = g->low_z[1];
    f.acc = g->frame_acc;
    f.count = g->frame_count;
    return f;
}

__device__ __forceinline__ void front_store(PulseStreamState *g, const FrontState &f) {
    g->band_z[0] = f.hz1;
    g->band_z[1] = f.hz2;
    g->band_z[2] = f.lz1;
    g->band_z[3] = f.lz2;
    g->low_z[0] = f.ez1;
    g->low_z[1] = f.ez2;
    g->frame_acc = f.acc;
    g->frame_count = f.count;
}

// one input sample x (already scaled); appends an energy value to my_new[np++] at a frame boundary
__device__ __forceinline__ void front_sample(const AudioFront &a, FrontState &f, float x, float *my_new, int &np) {
    const float y1 = a.band[0][0] * x + f.hz1;
    f.hz1 = a.band[0][1] * x - a.band[0][3] * y1 + f.hz2;
    f.hz2 = a.band[0][2] * x - a.band[0][4] * y1;
    const float y2 = a.band[1][0] * y1 + f.lz1;
    f.lz1 = a.band[1][1] * y1 - a.band[1][3] * y2 + f.lz2;
    f.lz2 = a.band[1][2] * y1 - a.band[1][4] * y2;
    f.acc += y2 * y2;
    f.count++;
    if (f.count >= a.frame_samples) {
        const float rms = sqrtf(f.acc / (float)a.frame_samples);
        const float e = a.low[0] * rms + f.ez1;
        f.ez1 = a.low[1] * rms - a.low[3] * e + f.ez2;
        f.ez2 = a.low[2] * rms - a.low[4] * e;
        my_new[np++] = e;
        f.acc = 0.f;
        f.count = 0;
    }
}

constexpr float PCM_TO_FLOAT = 1.f / 32767.f;  // audio_pulse_detector.cpp:100

}  // namespace sdrg
