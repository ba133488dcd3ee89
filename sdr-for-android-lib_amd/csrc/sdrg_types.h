// sdrg_types.h — POD state/parameter layouts shared by the host engine, the host design code and the
// HIP kernels.  No HIP includes, so plain g++ translation units can use it.
#pragma once

#include <stdint.h>

#include "../../include/sdrg.h"

namespace sdrg {

// ------------------------------------------------------------------------------------------------
// Per-stream FFTProcessor state (fft_process.h:57-109), one record per stream in HBM.  The stats kernel
// reads and updates it once per frame.
// ------------------------------------------------------------------------------------------------
struct StatsState {
    int64_t time_last_max_peak_ms;     // timeOfLastMaxPeak   (steady_clock, injected as ms)
    int64_t time_last_update_ms;       // timeOfLastMaxPeakUpdate
    float tracking_frequency;          // trackingFrequency
    float max_peak_db, max_peak_freq;  // maxPeakAndFrequency[0..1]
    int32_t max_peak_set;              // !maxPeakAndFrequency.empty()
    int32_t center_frequency_changed;  // sdr_bridge_internal::isCenterFrequencyChanged (per stream)
    int32_t peak_confirmed;
    int32_t det_buf[3];
    int32_t det_idx;
    int32_t detection_flag_sent;
    // getter-visible outputs; they keep their last value when a frame does not update them
    float mean_snr_db, mean_snr_sigma, peak_above_noise_mean_db, max_bin_snr_db, max_bin_snr_sigma;
    float best1khz_snr_db, best1khz_snr_sigma, best1khz_center_freq_hz, per_bin_mean;
    int32_t pad_;
};

// Window geometry of evaluateSignalStrength for one configuration (fft_process.cpp:124-216),
// computed on the host with the reference's float expressions; identical for every stream.
struct StatsGeometry {
    int32_t n;                 // sampCount
    int32_t focus_lo, focus_hi, focus_len;
    int32_t win_bins_1k;
    int32_t n_ref;             // reference windows collected (<= 10)
    int32_t win_lo[10], win_hi[10];
    int32_t max_pool;          // upper bound of pooled bins (sizes the LDS pool)
    int32_t span_lo, span_len; // bins [span_lo, span_lo + span_len) cover the focus and every window
    float freq_per_bin, nyquist;
    float cf_minus_nyq;        // static_cast<float>(centerFrequency) - nyquist   (:327)
    float cf_u32_minus_nyq;    // (centerFrequency - nyquist), uint32 promoted to float (:350)
    float cf_float;            // static_cast<float>(centerFrequency)
    int32_t cf_changed;        // setFrequency happened since the last frame (isCenterFrequencyChanged)
};

// ------------------------------------------------------------------------------------------------
// SSB chain.  processSSB_opt's statics (ssb_demod_opt.cpp:17-28, 223-282) are split in two:
// the parts every stream of an engine shares because every stream receives the same calls
// (mode globals, frozen frame size, filter coefficients: SsbControl, host-side) and the filter
// memories that depend on each stream's samples (SsbStreamState, HBM).
// ------------------------------------------------------------------------------------------------
struct SsbStreamState {
    float lpf_z1, lpf_z2;      // rfFilter.z1/z2 (:75-84), carried across frames
    float hp_z1, hp_z2;        // hp.z1/z2 (:177-186)
    float bp_z1, bp_z2;        // bp.z1/z2
    float pad_[2];
};

struct SsbParams {
    int32_t samp_count;        // frozen sampCount (:224-226)
    int32_t n_in;              // samples actually present per input frame (zero-pad above)
    int32_t upper;             // upperSideband
    int32_t decim;             // max(1, int(fs / 48000.0f))  (:273)
    int32_t n_taps;            // 255 or samp_count|1          (:122-123)
    int32_t pcm_len;           // outputs per frame
    float agc_target, agc_fast, agc_slow;
    float gain;                // demod_gain (floatToPCM)
    float transient_coeff;
    float lpf[5];              // a0 a1 a2 b1 b2 of rfFilter
    float hp[5];
    float bp[5];
};

}  // namespace sdrg
