// design.h — host-side filter design and window geometry (see design.cpp).
#pragma once

#include <stdint.h>

#include "sdrg_types.h"

namespace sdrg {

void design_lowpass(float fs, float fc, float Q, float c[5]);
void design_highpass(float fs, float f0, float Q, float c[5]);
void design_bandpass(float fs, float f0, float Q, float c[5]);
int design_fir(int64_t in_size, int decim, float cutoff_rel, float *h, int taps0 = 0);
int ssb_decim(uint32_t sample_rate);
int ssb_taps_for(int64_t samp_count, int taps0 = 0);
int ssb_pcm_len(int64_t samp_count, uint32_t sample_rate, int taps0 = 0);
uint32_t nco_increment(double hz, uint32_t sample_rate);
void nco_tables(float *tab);  // [2][1024][2] floats
// AudioPulseDetector::makeLP2 / makeHP2 (audio_pulse_detector.cpp:29-55), Q = 0.7071: {b0, b1, b2, a1, a2}
void design_pulse_sos(float fs, float fc, bool highpass, float c[5]);
StatsGeometry stats_geometry(uint32_t sample_rate, uint32_t center_frequency, int n, int focus_khz);

}  // namespace sdrg
