// sdrg_compat.hpp — source-compatible C++ drop-ins for the reference's internal DSP seams, implemented
// over the C ABI (sdrg.h).  A bridge that was written against
//
//   class FFTProcessor                       src/dsp/fft_process.h:29-55
//   void processSSB_opt(...)                  src/ssb/ssb_demod_opt.h:64-65
//
// compiles unchanged against these (include this header instead and `using namespace sdrg::compat;`),
// and its per-frame work then runs on the MI355X.  Each object owns a one-stream engine; the batched
// C ABI (sdrg_engine_process_device) is the high-throughput path for many receivers.
#pragma once

#include <complex>
#include <cstdint>
#include <functional>
#include <vector>

#include "sdrg.h"

namespace sdrg {
namespace compat {

// FftProcessorConfig (fft_process.h:20-26)
struct FftProcessorConfig {
    uint32_t centerFrequency;
    uint32_t sampleRate;
    int samplesPerReading;
    int freqFocusRangeKhz;
};

// FFTProcessor (fft_process.h:29-115): same public interface and getter semantics.  Frequency tracking
// uses std::chrono::steady_clock like the reference (fft_process.cpp:349-352).
class FFTProcessor {
public:
    FFTProcessor();
    ~FFTProcessor();
    FFTProcessor(const FFTProcessor &) = delete;
    FFTProcessor &operator=(const FFTProcessor &) = delete;

    void configure(const FftProcessorConfig &config);
    void process(const std::complex<float> *input_buf, uint32_t input_len);
    // setFrequency (sdr-bridge-java-soapy.cpp:907) raises isCenterFrequencyChanged; call this instead
    void notifyCenterFrequencyChanged();

    const std::vector<float> &getPowerSpectrum() const { return power_shifted_vec_; }
    float getMeanSnrDb() const { return rec_.mean_snr_db; }
    float getMeanSnrSigma() const { return rec_.mean_snr_sigma; }
    long getTrackingFrequency() const { return static_cast<long>(rec_.tracking_frequency); }
    int getDetectionFlag() const { return rec_.detection_flag; }
    float getPeakAboveNoiseMeanDb() const { return rec_.peak_above_noise_mean_db; }
    float getMaxBinSnrDb() const { return rec_.max_bin_snr_db; }
    float getMaxBinSnrSigma() const { return rec_.max_bin_snr_sigma; }
    float getBest1kHzSnrDb() const { return rec_.best1khz_snr_db; }
    float getBest1kHzSnrSigma() const { return rec_.best1khz_snr_sigma; }
    float getBest1kHzCenterFreqHz() const { return rec_.best1khz_center_freq_hz; }
    float getPerBinMean() const { return rec_.per_bin_mean; }

    // status of the last call (the reference never fails; the engine can, e.g. without a GPU)
    int32_t lastStatus() const { return status_; }
    // process with an explicit clock (ms) instead of steady_clock, for reproducible tests
    void processAt(const std::complex<float> *input_buf, uint32_t input_len, int64_t now_ms);

private:
    sdrg_engine *eng_ = nullptr;
    sdrg_config cfg_{};
    bool configured_ = false;
    bool cf_changed_ = false;
    int32_t status_ = SDRG_OK;
    std::vector<float> power_shifted_vec_;
    sdrg_frame_record rec_{};
};

// processSSB_opt (ssb_demod_opt.h:64-65).  Like the reference, the chain's filter state is process-global
// (one shared one-stream engine); `pulse` is left untouched as in the reference (its detector is a TO DO).
void processSSB_opt(std::vector<std::complex<float>> iq, uint32_t sampleRate, bool upperSideband,
                    std::vector<int16_t> &pcmOut, bool &pulse, int mode);

// Status of the last processSSB_opt call.
int32_t lastSsbStatus();

class AudioPulseDetector;

// SSBProcessor (src/ssb/ssb_processor.h:24-58): the worker thread + 3-deep drop-oldest queue, over
// sdrg_ssb_processor (frames run through a one-stream engine's SSB + audio-pulse stages).  The sound mode the
// reference reads from BridgeConfig per frame is set here with setSoundMode.
using PcmDataCallback = std::function<void(const std::vector<int16_t> &)>;
class SSBProcessor {
public:
    SSBProcessor();
    ~SSBProcessor();
    SSBProcessor(const SSBProcessor &) = delete;
    SSBProcessor &operator=(const SSBProcessor &) = delete;

    void startProcessing(PcmDataCallback pcm_cb);
    void startProcessing(PcmDataCallback pcm_cb, std::function<void(float, int)> pulse_cb);
    void stopProcessing();
    void enqueueData(std::vector<std::complex<float>> &&iq_data, uint32_t sample_rate);
    void setPulseConfig(const sdrg_pulse_config &cfg);
    float getAmbientEnergy() const;
    float getCurrentRatio() const { return 0.f; }
    void setSoundMode(int mode);
    int32_t lastStatus() const { return status_; }

private:
    static void onPcm(void *u, const int16_t *p, int32_t n);
    static void onPulse(void *u, float strength, int32_t live_etat);
    sdrg_ssb_processor *proc_ = nullptr;
    PcmDataCallback pcm_cb_;
    std::function<void(float, int)> pulse_cb_;
    std::vector<int16_t> pcm_;
    int32_t status_ = SDRG_OK;
};

// SpectralPulseDetector (src/dsp/spectral_pulse_detector.h:19-79) and AudioPulseDetector
// (src/ssb/audio_pulse_detector.h:15-104): same public interface; each object owns a one-stream
// sdrg_pulse_bank, so its state machine runs in the GPU kernels (csrc/pulse.hip).
enum class PulseLevel { NONE = 0, LOW = 1, MEDIUM = 2, STRONG = 3 };

class SpectralPulseDetector {
public:
    using PulseLevel = compat::PulseLevel;
    struct Config {  // spectral_pulse_detector.h:23-35
        float fsEnergy = 20.f, zDefaultS = 0.666f, tTargetInit = 1.75f, dtTolS = 0.150f;
        float snrMin = 1.5f, snrRhythm = 2.5f, snrStrong = 4.0f, dispersionMax = 1.3f;
        int sumNMax = 7;
        float liveWindowT = 4.0f, liveDivisor = 3.0f;
    };
    SpectralPulseDetector() : SpectralPulseDetector(Config{}) {}
    explicit SpectralPulseDetector(const Config &cfg);
    ~SpectralPulseDetector();
    SpectralPulseDetector(const SpectralPulseDetector &) = delete;
    SpectralPulseDetector &operator=(const SpectralPulseDetector &) = delete;

    void configure(const Config &cfg);
    PulseLevel process(float snrSigma, float freqHz);
    PulseLevel pulseDetected() const { return static_cast<PulseLevel>(out_.level); }
    float lastPulseStrength() const { return out_.strength; }
    bool isLocked() const { return out_.locked != 0; }
    float lockedPeriodS() const { return out_.period_s; }
    int liveEtat() const { return out_.live_etat; }
    float estimatedFreqHz() const { return out_.est_freq_hz; }
    void reset();
    int32_t lastStatus() const { return status_; }

private:
    sdrg_pulse_bank *bank_ = nullptr;
    sdrg_pulse_output out_{};
    float t_target_init_ = 1.75f;
    int32_t status_ = SDRG_OK;
};

class AudioPulseDetector {
public:
    using PulseLevel = compat::PulseLevel;
    struct Config {  // audio_pulse_detector.h:19-37
        float sampleRate = 48000.f, fMin = 1500.f, fMax = 4000.f, fsEnergy = 100.f, smoothCutoff = 5.f;
        float zDefaultS = 0.666f, tTargetInit = 1.75f, dtTolS = 0.150f;
        float snrMin = 1.0f, snrRhythm = 1.1f, snrStrong = 2.0f, dispersionMax = 1.3f;
        int sumNMax = 7;
        float liveWindowT = 4.0f, liveDivisor = 3.0f;
        int noiseRefFar = 80, noiseRefNear = 40;
    };
    AudioPulseDetector() : AudioPulseDetector(Config{}) {}
    explicit AudioPulseDetector(const Config &cfg);
    ~AudioPulseDetector();
    AudioPulseDetector(const AudioPulseDetector &) = delete;
    AudioPulseDetector &operator=(const AudioPulseDetector &) = delete;

    PulseLevel process(const std::vector<float> &audio);
    PulseLevel process(const std::vector<int16_t> &pcm);
    PulseLevel pulseDetected() const { return static_cast<PulseLevel>(out_.level); }
    float lastPulseStrength() const { return out_.strength; }
    bool isLocked() const { return out_.locked != 0; }
    float lockedPeriodS() const { return out_.period_s; }
    int liveEtat() const { return out_.live_etat; }
    void reset();
    int32_t lastStatus() const { return status_; }

private:
    PulseLevel run(const void *samples, int fmt, size_t n);
    sdrg_pulse_bank *bank_ = nullptr;
    sdrg_pulse_output out_{};
    float t_target_init_ = 1.75f;
    int32_t status_ = SDRG_OK;
};

}  // namespace compat
}  // namespace sdrg
