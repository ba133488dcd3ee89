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
    if ((uint32_t)cfg_.samples_per_reading != input_len) {  // process() takes whatever length it is handed
        cfg_.samples_per_reading = (int32_t)input_len;
        if (eng_) {
            status_ = sdrg_engine_set_samples_per_reading(eng_, (int32_t)input_len);
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

// ---- SSBProcessor (ssb_processor.cpp:26-115) ------------------------------------------------------------
SSBProcessor::SSBProcessor() {
    status_ = sdrg_ssb_processor_create(0, 0, &proc_);
    if (status_) proc_ = nullptr;
}

SSBProcessor::~SSBProcessor() {
    if (proc_) sdrg_ssb_processor_destroy(proc_);  // stopProcessing() first, as the reference's destructor
}

void SSBProcessor::onPcm(void *u, const int16_t *p, int32_t n) {
    SSBProcessor *s = static_cast<SSBProcessor *>(u);
    if (!s->pcm_cb_) return;
    s->pcm_.assign(p, p + n);
    s->pcm_cb_(s->pcm_);
}

void SSBProcessor::onPulse(void *u, float strength, int32_t live_etat) {
    SSBProcessor *s = static_cast<SSBProcessor *>(u);
    if (s->pulse_cb_) s->pulse_cb_(strength, live_etat);
}

void SSBProcessor::startProcessing(PcmDataCallback pcm_cb) { startProcessing(std::move(pcm_cb), nullptr); }

void SSBProcessor::startProcessing(PcmDataCallback pcm_cb, std::function<void(float, int)> pulse_cb) {
    if (!proc_) return;
    pcm_cb_ = std::move(pcm_cb);
    pulse_cb_ = std::move(pulse_cb);
    const sdrg_ssb_callbacks c{this, &SSBProcessor::onPcm, &SSBProcessor::onPulse};
    status_ = sdrg_ssb_processor_start(proc_, &c);
}

void SSBProcessor::stopProcessing() {
    if (proc_) status_ = sdrg_ssb_processor_stop(proc_);
}

void SSBProcessor::enqueueData(std::vector<std::complex<float>> &&iq_data, uint32_t sample_rate) {
    if (!proc_ || iq_data.empty()) return;
    status_ = sdrg_ssb_processor_enqueue(proc_, iq_data.data(), SDRG_IQ_CF32, (int32_t)iq_data.size(), sample_rate);
}

void SSBProcessor::setPulseConfig(const sdrg_pulse_config &cfg) {
    if (proc_) status_ = sdrg_ssb_processor_set_pulse_config(proc_, &cfg);
}

float SSBProcessor::getAmbientEnergy() const { return proc_ ? sdrg_ssb_processor_get_ambient_energy(proc_) : 0.f; }

void SSBProcessor::setSoundMode(int mode) {
    if (proc_) status_ = sdrg_ssb_processor_set_sound_mode(proc_, mode);
}

// ---- pulse detectors ------------------------------------------------------------------------------
namespace {

sdrg_pulse_config spectral_cfg(const SpectralPulseDetector::Config &c) {
    sdrg_pulse_config p;
    sdrg_pulse_config_default(SDRG_PULSE_SPECTRAL, &p);
    p.fs_energy = c.fsEnergy;
    p.z_default_s = c.zDefaultS;
    p.t_target_init = c.tTargetInit;
    p.dt_tol_s = c.dtTolS;
    p.snr_min = c.snrMin;
    p.snr_rhythm = c.snrRhythm;
    p.snr_strong = c.snrStrong;
    p.dispersion_max = c.dispersionMax;
    p.sum_n_max = c.sumNMax;
    p.live_window_t = c.liveWindowT;
    p.live_divisor = c.liveDivisor;
    return p;
}

sdrg_pulse_config audio_cfg(const AudioPulseDetector::Config &c) {
    sdrg_pulse_config p;
    sdrg_pulse_config_default(SDRG_PULSE_AUDIO, &p);
    p.sample_rate = c.sampleRate;
    p.f_min = c.fMin;
    p.f_max = c.fMax;
    p.fs_energy = c.fsEnergy;
    p.smooth_cutoff = c.smoothCutoff;
    p.z_default_s = c.zDefaultS;
    p.t_target_init = c.tTargetInit;
    p.dt_tol_s = c.dtTolS;
    p.snr_min = c.snrMin;
    p.snr_rhythm = c.snrRhythm;
    p.snr_strong = c.snrStrong;
    p.dispersion_max = c.dispersionMax;
    p.sum_n_max = c.sumNMax;
    p.live_window_t = c.liveWindowT;
    p.live_divisor = c.liveDivisor;
    p.noise_ref_far = c.noiseRefFar;
    p.noise_ref_near = c.noiseRefNear;
    return p;
}

void fresh_output(sdrg_pulse_output &o, float t_target_init) {
    std::memset(&o, 0, sizeof(o));
    o.period_s = t_target_init;
}

}  // namespace

SpectralPulseDetector::SpectralPulseDetector(const Config &cfg) : t_target_init_(cfg.tTargetInit) {
    const sdrg_pulse_config p = spectral_cfg(cfg);
    status_ = sdrg_pulse_bank_create(SDRG_PULSE_SPECTRAL, &p, 1, 0, &bank_);
    if (status_) bank_ = nullptr;
    fresh_output(out_, t_target_init_);
}

SpectralPulseDetector::~SpectralPulseDetector() {
    if (bank_) sdrg_pulse_bank_destroy(bank_);
}

// configure (spectral_pulse_detector.cpp:6-8): the config only; tTarget_ and the history are kept
void SpectralPulseDetector::configure(const Config &cfg) {
    const sdrg_pulse_config p = spectral_cfg(cfg);
    if (bank_) status_ = sdrg_pulse_bank_configure(bank_, &p);
}

SpectralPulseDetector::PulseLevel SpectralPulseDetector::process(float snrSigma, float freqHz) {
    if (!bank_) return pulseDetected();
    status_ = sdrg_pulse_bank_process_spectral_host(bank_, &snrSigma, &freqHz, &out_);
    return pulseDetected();
}

void SpectralPulseDetector::reset() {
    if (bank_) status_ = sdrg_pulse_bank_reset(bank_);
    sdrg_pulse_config c;
    if (bank_ && sdrg_pulse_bank_get_config(bank_, &c) == SDRG_OK) t_target_init_ = c.t_target_init;
    fresh_output(out_, t_target_init_);
}

AudioPulseDetector::AudioPulseDetector(const Config &cfg) : t_target_init_(cfg.tTargetInit) {
    const sdrg_pulse_config p = audio_cfg(cfg);
    status_ = sdrg_pulse_bank_create(SDRG_PULSE_AUDIO, &p, 1, 0, &bank_);
    if (status_) bank_ = nullptr;
    fresh_output(out_, t_target_init_);
}

AudioPulseDetector::~AudioPulseDetector() {
    if (bank_) sdrg_pulse_bank_destroy(bank_);
}

AudioPulseDetector::PulseLevel AudioPulseDetector::run(const void *samples, int fmt, size_t n) {
    if (!bank_) return pulseDetected();
    status_ = sdrg_pulse_bank_process_audio_host(bank_, samples, fmt, (int32_t)n, &out_);
    return pulseDetected();
}

AudioPulseDetector::PulseLevel AudioPulseDetector::process(const std::vector<float> &audio) {
    return run(audio.data(), 1, audio.size());
}

AudioPulseDetector::PulseLevel AudioPulseDetector::process(const std::vector<int16_t> &pcm) {
    return run(pcm.data(), 0, pcm.size());
}

void AudioPulseDetector::reset() {
    if (bank_) status_ = sdrg_pulse_bank_reset(bank_);
    fresh_output(out_, t_target_init_);
}

}  // namespace compat
}  // namespace sdrg
