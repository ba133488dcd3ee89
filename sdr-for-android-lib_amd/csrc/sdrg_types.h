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
    float log_focus_len;       // std::log(static_cast<float>(focusLen)) (:282) with glibc's logf, on the host
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
    // NCO/short-FIR variant (a build extension, sdrg_engine_set_ssb_variant): when nco_on, sample t of the
    // frame is the real part of (I + jQ) e^{-j 2 pi ph / 2^32}, ph = nco_phase + nco_inc * t (mod 2^32),
    // with the phasor from the two-level table nco_tab (design.cpp nco_tables); samples past n_in stay 0
    int32_t nco_on;
    uint32_t nco_inc, nco_phase;
    const float *nco_tab;      // device [2][1024] {re, im}
};

// ------------------------------------------------------------------------------------------------
// Beacon pulse detectors (SpectralPulseDetector / AudioPulseDetector).  The reference's std::deque members
// become per-stream rings in HBM of `cap` slots (a power of two >= maxBuf + 8): eBuf_ / freqBuf_ and the
// ROI list, addressed as slot (head + logical index) & (cap - 1); the small bounded deques (last3Dts_,
// histDts_, histN_) live in the state record itself, and the 30-entry freqHistory_ in a 32-slot ring.
// ------------------------------------------------------------------------------------------------
constexpr int PULSE_FH_SLOTS = 32;  // freqHistory_ ring (kFreqHistoryMax = 30, spectral_pulse_detector.h:67)

struct PulseStreamState {
    double ols_a, ols_b;       // estimatedFreqHz regression f = a t + b over freqHistory_ (recomputed per ROI)
    uint32_t head;             // ring slot of eBuf_[0]
    int32_t n;                 // eBuf_.size()
    float t0;                  // eBufT0_
    int32_t last_scan;         // lastScanIdx_
    float t_last_roi;          // tLastRoi_
    int32_t locked;            // isLocked_
    float t_target;            // tTarget_
    int32_t live_etat;         // liveEtat_
    float last_snr;            // lastSnr_
    int32_t level;             // lastLevel_
    uint32_t roi_head;         // ring slot of rois_[0]
    int32_t n_rois;
    int32_t n_last3, n_hist;
    float last3[3];            // last3Dts_
    float hist_dts[5];         // histDts_
    int32_t hist_n[5];         // histN_
    int32_t fh_head, n_fh;     // freqHistory_ ring
    int32_t ols_mode;          // 0: < 2 samples (0 Hz), 1: degenerate (mean), 2: a t + b
    float ols_mean;            // (float)(sum_f / n) for mode 1
    int32_t overflow;          // ROI ring overflows (diagnostic; never within the documented bound)
    float band_z[4];           // audio: band-pass SOS z1/z2 (HP, LP)
    float low_z[2];            // audio: energy low-pass z1/z2
    int32_t frame_count;       // audio: frameCount_
    float frame_acc;           // audio: frameAcc_
    int32_t pad_[2];
};

struct PulseParams {
    int32_t cap_mask;          // ring slots - 1
    int32_t max_buf;           // (int)(10.f * fsEnergy)   (spectral :31, audio :118)
    float fs_energy, inv_fs;   // fsEnergy, 1.f / fsEnergy (the eBufT0_ increment)
    float z_default_s, dt_tol_s, snr_min, snr_rhythm, snr_strong, dispersion_max;
    int32_t sum_n_max;
    float live_window_t, live_divisor;
    int32_t noise_far, noise_near;
    int32_t frame_samples;     // audio: max(1, (int)(sampleRate / fsEnergy))
    float band[2][5];          // audio: HP(fMin), LP(fMax) b0 b1 b2 a1 a2
    float low[5];              // audio: LP(smoothCutoff) at fsEnergy
};

// The audio detector's front end as the SSB kernels run it on the PCM they produce (band-pass, RMS per
// energy frame, energy low-pass): its coefficients, the per-stream state records (only the front-end
// fields are touched) and where the energy values of the call go ([n_streams][max_new], counts).
struct AudioFront {
    float band[2][5];
    float low[5];
    int32_t frame_samples;
    int32_t max_new;
    PulseStreamState *state;
    float *new_e;
    int32_t *new_count;
};

}  // namespace sdrg
