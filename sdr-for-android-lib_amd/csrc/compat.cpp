// compat.cpp — FFTProcessor / processSSB_opt drop-ins (include/sdrg_compat.hpp) over the C ABI.
#include "../../include/sdrg_compat.hpp"

#include <chrono>
#include <cstring>
#include <mutex>

namespace sdrg {
namespace compat {

namespace {

int64_t steady_ms() {
    return std::chrono::duration_cast<std::chrono::milliseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

sdrg_config make_config(uint32_t cf, uint32_t fs, int n, int focus_khz, int mode) {
    sdrg_config c{};
    c.center_frequency = cf;
    c.sample_rate = fs;
    c.samples_per_reading = n;
    c.freq_focus_range_khz = focus_khz;
    c.gain = 0;
    c.sound_mode = mode;
    c.refresh_fft_ms = 50;
    c.refresh_peak_ms = 200;
    c.refresh_signal_strength_ms = 30;
    return c;
}

}  // namespace

FFTProcessor::FFTProcessor() = default;

FFTProcessor::~FFTProcessor() {
    if (eng_) sdrg_engine_destroy(eng_);
}

// FFTProcessor::configure (fft_process.cpp:20-39)
void FFTProcessor::configure(const FftProcessorConfig &config) {
    cfg_ = make_config(config.centerFrequency, config.sampleRate, config.samplesPerReading,
                       config.freqFocusRangeKhz, 1);
    configured_ = true;
    if (eng_) status_ = sdrg_engine_apply_config(eng_, &cfg_);
}

void FFTProcessor::notifyCenterFrequencyChanged() {
    cf_changed_ = true;
}

void FFTProcessor::process(const std::complex<float> *input_buf, uint32_t input_len) {
    processAt(input_buf, input_len, steady_ms());
}

// FFTProcessor::process (fft_process.cpp:42-105): the frame length is the call's input_len, as in the
// reference (which re-plans FFTW for whatever length it receives).
void FFTProcessor::processAt(const std::complex<float> *input_buf, uint32_t input_len, int64_t now_ms) {
    if (!configured_) cfg_ = make_config(0, 2500000, (int)input_len, 5, 1);
    if ((uint32_t)cfg_.samples_per_reading != input_len) {
        cfg_.samples_per_reading = (int32_t)input_len;
        if (eng_) {
            status_ = sdrg_engine_apply_config(eng_, &cfg_);
            if (status_) return;
        }
    }
    if (!eng_) {
        status_ = sdrg_engine_create(&cfg_, 1, 0, &eng_);
        if (status_) {
            eng_ = nullptr;
            return;
        }
    }
    if (cf_changed_) {
        status_ = sdrg_engine_set_frequency(eng_, cfg_.center_frequency);
        if (status_) return;
        cf_changed_ = false;
    }
    power_shifted_vec_.resize(input_len);
    status_ = sdrg_engine_process_host(eng_, input_buf, SDRG_IQ_CF32, SDRG_STAGE_SPECTRUM | SDRG_STAGE_STATS,
                                       power_shifted_vec_.data(), &rec_, nullptr, now_ms);
}

namespace {
std::mutex g_ssb_mu;
sdrg_engine *g_ssb = nullptr;
sdrg_config g_ssb_cfg{};
int32_t g_ssb_status = SDRG_OK;
}  // namespace

int32_t lastSsbStatus() {
    std::lock_guard<std::mutex> lk(g_ssb_mu);
    return g_ssb_status;
}

// processSSB_opt (ssb_demod_opt.cpp:221-296): function-static state -> one process-global engine.
void processSSB_opt(std::vector<std::complex<float>> iq, uint32_t sampleRate, bool upperSideband,
                    std::vector<int16_t> &pcmOut, bool &pulse, int mode) {
    (void)pulse;
    std::lock_guard<std::mutex> lk(g_ssb_mu);
    const int n = (int)iq.size();
    if (!g_ssb) {
        g_ssb_cfg = make_config(0, sampleRate, n, 5, mode);
        g_ssb_status = sdrg_engine_create(&g_ssb_cfg, 1, 0, &g_ssb);
        if (g_ssb_status) {
            g_ssb = nullptr;
            pcmOut.clear();
            return;
        }
    } else if (g_ssb_cfg.samples_per_reading != n || (uint32_t)g_ssb_cfg.sample_rate != sampleRate ||
               g_ssb_cfg.sound_mode != mode) {
        g_ssb_cfg.samples_per_reading = n;
        g_ssb_cfg.sample_rate = sampleRate;
        g_ssb_cfg.sound_mode = mode;
        g_ssb_status = sdrg_engine_apply_config(g_ssb, &g_ssb_cfg);
        if (g_ssb_status) {
            pcmOut.clear();
            return;
        }
    }
    g_ssb_status = sdrg_engine_set_upper_sideband(g_ssb, upperSideband ? 1 : 0);
    if (g_ssb_status) return;
    pcmOut.resize((size_t)sdrg_engine_pcm_len(g_ssb));
    g_ssb_status = sdrg_engine_process_host(g_ssb, iq.data(), SDRG_IQ_CF32, SDRG_STAGE_SSB, nullptr, nullptr,
                                            pcmOut.empty() ? nullptr : pcmOut.data(), 0);
    if (g_ssb_status) pcmOut.clear();
}

}  // namespace compat
}  // namespace sdrg
