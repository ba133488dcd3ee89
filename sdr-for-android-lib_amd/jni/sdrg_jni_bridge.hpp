// sdrg_jni_bridge.hpp — the SDRBridge JNI surface of the reference (src/sdr-bridge-java-soapy.cpp:625-1171)
// over the engine's C ABI, written once against a JNI "traits" type so the same logic runs under the real
// JNIEnv (sdrg_jni.cpp, built with the Android NDK's jni.h) and under a recording fake in the tests
// (tests/cpp/jni_bridge_test.cpp) — there is no JVM in this image.
//
// What it replaces, per reference function:
//   applyConfig(9 SDRConfig fields)  :1073-1141  -> sdrg_engine_create / _apply_config (+ the spectral pulse
//                                                    detector's fsEnergy, done by the engine)
//   read(12 callbacks)               :625-764    -> global refs + "invoke" method IDs with the reference's
//                                                    signatures; frames then arrive through onFrame()
//   soapyCallback(buf, len)          :424-493    -> onFrame(): enqueue the frame for the SSB worker (:441-442),
//                                                    then one engine call for FFT + stats + spectral pulse
//   SSB worker loop                  ssb_processor.cpp:26-115 -> sdrg_ssb_processor (3-deep drop-oldest queue,
//                                                    worker thread); pcm and audioPulse callbacks on that
//                                                    thread, attached to the JVM per call (:697-760)
//                                    (SsbMode::SYNCHRONOUS instead runs SSB + audio pulse in the frame's engine
//                                    call and calls back after soapyCallback's callbacks: deterministic, no drops)
//   stopReading / close              :766-876    -> SSB worker stopped, callbacks dropped / global refs deleted,
//                                                    engines destroyed
//   setFrequency / setFrequencyFocusRange         -> engine setters (FFTProcessor::configure + the flag)
//   setSampleRate / setSamplesPerReading (:931-1021) -> BridgeConfig only: sdrg_engine_set_sample_rate /
//                                                    _set_samples_per_reading (the spectral pulse detector and
//                                                    the statistics' configured rate are left alone)
//   setSoundMode / setRefresh*Ms     :1042-1071  -> sound mode of both halves / stored only
//   setPulseConfig                   :1143-1161  -> no-op, as in the reference
//   getAmbientAudioEnergy / getCurrentAudioRatio :1163-1171 -> lastPulseStrength() / 0
// Device I/O (initDongle, getDriver, tuner gains and ranges) stays with SoapySDR and is not part of this.
#pragma once

#include <algorithm>
#include <complex>
#include <cstdint>
#include <mutex>
#include <vector>

#include "../../include/sdrg.h"

namespace sdrg {
namespace jni {

// J must provide: types Env, Obj, Mid, Vm; NewGlobalRef, DeleteGlobalRef, MethodOf(env, obj, sig) ("invoke"),
// ClearException(env); CallF / CallI / CallJ / CallFF / CallFI / CallFIJ / CallFloats / CallShorts;
// VmOf(env), and Attach(vm, &attached) / Detach(vm) for the SSB worker thread (GetEnv / AttachCurrentThread).
template <class J>
class Bridge {
public:
    using Env = typename J::Env;
    using Obj = typename J::Obj;
    using Mid = typename J::Mid;
    using Vm = typename J::Vm;
    enum class SsbMode { QUEUED, SYNCHRONOUS };
    enum Callback {
        FFT, DETECTION_FLAG, MEAN_SNR, MEAN_SNR_SIGMA, PEAK_FREQUENCY, PCM, AUDIO_PULSE, PEAK_ABOVE_NOISE_MEAN,
        MAX_BIN, BEST_1KHZ, SPECTRAL_PULSE, NOISE_LEVEL, N_CALLBACKS
    };
    static constexpr const char *kSignature[N_CALLBACKS] = {"([F)V", "(I)V", "(F)V", "(F)V", "(J)V", "([S)V",
                                                             "(FI)V", "(F)V", "(FF)V", "(FF)V", "(FIJ)V", "(F)V"};

    ~Bridge() {
        if (ssb_) sdrg_ssb_processor_destroy(ssb_);
        if (eng_) sdrg_engine_destroy(eng_);
    }

    // QUEUED (default, the reference's SSBProcessor) or SYNCHRONOUS; set before read()
    void setSsbMode(SsbMode m) { mode_ = m; }

    bool applyConfig(Env *, int64_t centerFrequency, int64_t sampleRate, int32_t samplesPerReading,
                     int32_t freqFocusRangeKhz, int32_t gain, int64_t refreshFFTMs, int64_t refreshPeakMs,
                     int64_t refreshSignalStrengthMs, int32_t soundMode) {
        cfg_ = sdrg_config{centerFrequency, sampleRate, samplesPerReading, freqFocusRangeKhz, gain, soundMode,
                           refreshFFTMs, refreshPeakMs, refreshSignalStrengthMs};
        status_ = eng_ ? sdrg_engine_apply_config(eng_, &cfg_) : sdrg_engine_create(&cfg_, 1, 0, &eng_);
        if (status_ != SDRG_OK && !eng_) return false;
        return status_ == SDRG_OK;  // the reference returns false only when a device call throws (:1115-1118)
    }

    // read(): the 12 callback objects in the reference's parameter order (:625-640)
    void read(Env *env, const Obj (&cbs)[N_CALLBACKS]) {
        if (ssb_) sdrg_ssb_processor_stop(ssb_);  // the worker reads the callback table
        dropCallbacks(env);
        for (int i = 0; i < N_CALLBACKS; i++) {
            if (!cbs[i]) continue;
            cb_[i].obj = J::NewGlobalRef(env, cbs[i]);
            cb_[i].mid = J::MethodOf(env, cbs[i], kSignature[i]);
        }
        vm_ = J::VmOf(env);
        if (mode_ == SsbMode::QUEUED) {  // ssbProcessor.startProcessing(pcm lambda, pulse lambda) (:694-760)
            if (!ssb_ && (status_ = sdrg_ssb_processor_create(0, 0, &ssb_)) != SDRG_OK) {
                ssb_ = nullptr;
                return;
            }
            sdrg_ssb_processor_set_sound_mode(ssb_, cfg_.sound_mode);
            const sdrg_ssb_callbacks c{this, &Bridge::pcmFromWorker, &Bridge::pulseFromWorker};
            status_ = sdrg_ssb_processor_start(ssb_, &c);
        }
        reading_ = true;
    }

    // One exact-N frame of CF32 samples (the rx_process_thread's chunk, :590-615); now_ms is the clock the
    // reference reads from steady_clock for its 300 ms tracking latch (fft_process.cpp:333-361).
    void onFrame(Env *env, const std::complex<float> *buf, uint32_t len, int64_t now_ms) {
        if (!eng_ || !reading_ || !buf || len == 0) return;
        if ((uint32_t)cfg_.samples_per_reading != len) {  // the reference processes whatever len it is handed
            cfg_.samples_per_reading = (int32_t)len;
            if ((status_ = sdrg_engine_set_samples_per_reading(eng_, (int32_t)len)) != SDRG_OK) return;
        }
        const bool queued = mode_ == SsbMode::QUEUED && ssb_;
        if (queued) {  // ssbProcessor.enqueueData(copy of buf, BridgeConfig sampleRate) (:441-442)
            status_ = sdrg_ssb_processor_enqueue(ssb_, buf, SDRG_IQ_CF32, (int32_t)len, cfg_.sample_rate);
            if (status_ != SDRG_OK) return;
        }
        spec_.resize(len);
        pcm_.resize(queued ? 0 : (size_t)std::max(0, sdrg_engine_pcm_len(eng_)));
        const int32_t stages = queued ? SDRG_STAGE_SPECTRUM | SDRG_STAGE_STATS | SDRG_STAGE_SPECTRAL_PULSE : SDRG_STAGE_ALL;
        status_ = sdrg_engine_process_host(eng_, buf, SDRG_IQ_CF32, stages, spec_.data(), &rec_,
                                           pcm_.empty() ? nullptr : pcm_.data(), now_ms);
        if (status_ != SDRG_OK) return;  // nothing throws across JNI: the frame is dropped
        if ((status_ = sdrg_engine_get_pulse_outputs(eng_, &spectral_, queued ? nullptr : &audio_)) != SDRG_OK) return;
        // soapyCallback (:458-488)
        if (has(FFT)) J::CallFloats(env, cb_[FFT].obj, cb_[FFT].mid, spec_.data(), (int32_t)len);
        if (has(DETECTION_FLAG)) J::CallI(env, cb_[DETECTION_FLAG].obj, cb_[DETECTION_FLAG].mid, rec_.detection_flag);
        if (has(MEAN_SNR)) J::CallF(env, cb_[MEAN_SNR].obj, cb_[MEAN_SNR].mid, rec_.mean_snr_db);
        if (has(MEAN_SNR_SIGMA)) J::CallF(env, cb_[MEAN_SNR_SIGMA].obj, cb_[MEAN_SNR_SIGMA].mid, rec_.mean_snr_sigma);
        if (has(PEAK_FREQUENCY)) J::CallJ(env, cb_[PEAK_FREQUENCY].obj, cb_[PEAK_FREQUENCY].mid, rec_.tracking_frequency);
        if (has(PEAK_ABOVE_NOISE_MEAN))
            J::CallF(env, cb_[PEAK_ABOVE_NOISE_MEAN].obj, cb_[PEAK_ABOVE_NOISE_MEAN].mid, rec_.peak_above_noise_mean_db);
        if (has(MAX_BIN)) J::CallFF(env, cb_[MAX_BIN].obj, cb_[MAX_BIN].mid, rec_.max_bin_snr_db, rec_.max_bin_snr_sigma);
        if (has(BEST_1KHZ))
            J::CallFF(env, cb_[BEST_1KHZ].obj, cb_[BEST_1KHZ].mid, rec_.best1khz_snr_db, rec_.best1khz_snr_sigma);
        if (has(NOISE_LEVEL)) J::CallF(env, cb_[NOISE_LEVEL].obj, cb_[NOISE_LEVEL].mid, rec_.per_bin_mean);
        if (has(SPECTRAL_PULSE))
            J::CallFIJ(env, cb_[SPECTRAL_PULSE].obj, cb_[SPECTRAL_PULSE].mid, spectral_.input, spectral_.live_etat,
                       spectral_.est_freq_hz_rounded);
        // SYNCHRONOUS: the SSB worker's calls (ssb_processor.cpp:105-113) right here: pcm only when the frame
        // produced samples, pulse always
        if (!queued) {
            if (has(PCM) && !pcm_.empty()) J::CallShorts(env, cb_[PCM].obj, cb_[PCM].mid, pcm_.data(), (int32_t)pcm_.size());
            if (has(AUDIO_PULSE)) J::CallFI(env, cb_[AUDIO_PULSE].obj, cb_[AUDIO_PULSE].mid, audio_.strength, audio_.live_etat);
        }
        J::ClearException(env);
    }

    // stopReading (:766-793): the rx side stops, then ssbProcessor.stopProcessing()
    void stopReading(Env *) {
        reading_ = false;
        if (ssb_) sdrg_ssb_processor_stop(ssb_);
    }

    // two-phase stop for callers that serialise the bridge behind a lock (LockedBridge below): under the lock,
    // stop reading and hand out the SSB processor; the caller stops (joins) it after releasing the lock, so
    // callbacks running on the worker can still enter the bridge
    sdrg_ssb_processor *beginStopReading() {
        reading_ = false;
        return ssb_;
    }
    sdrg_ssb_processor *ssbHandle() const { return ssb_; }
    // close(), first phase: the processor leaves the bridge (the caller destroys it outside the lock)
    sdrg_ssb_processor *detachSsb() {
        reading_ = false;
        sdrg_ssb_processor *p = ssb_;
        ssb_ = nullptr;
        return p;
    }

    void close(Env *env) {
        reading_ = false;
        if (ssb_) sdrg_ssb_processor_destroy(ssb_);
        ssb_ = nullptr;
        dropCallbacks(env);  // every global ref, noiseLevel's included (the reference leaks that one, :826-874)
        if (eng_) sdrg_engine_destroy(eng_);
        eng_ = nullptr;
    }

    // test / shutdown helper: wait until the SSB worker has processed what is queued
    void drainSsb() {
        if (ssb_) sdrg_ssb_processor_drain(ssb_);
    }
    // SSB frames enqueued / dropped (queue full) / processed so far (QUEUED mode)
    void ssbCounters(int64_t *enq, int64_t *drop, int64_t *proc) const {
        *enq = *drop = *proc = 0;
        if (ssb_) sdrg_ssb_processor_counters(ssb_, enq, drop, proc, nullptr);
    }

    void setFrequency(Env *, int64_t hz) {
        cfg_.center_frequency = hz;
        if (eng_) status_ = sdrg_engine_set_frequency(eng_, hz);  // raises isCenterFrequencyChanged (:907)
    }
    // BridgeConfig only (:931-953, :1015-1021): no FFTProcessor::configure, no spectral pulse reconfiguration
    void setSampleRate(Env *, int64_t fs) {
        cfg_.sample_rate = fs;
        if (eng_) status_ = sdrg_engine_set_sample_rate(eng_, fs);
    }
    void setSamplesPerReading(Env *, int32_t n) {
        cfg_.samples_per_reading = n;
        if (eng_) status_ = sdrg_engine_set_samples_per_reading(eng_, n);
    }
    void setFrequencyFocusRange(Env *, int32_t khz) {
        cfg_.freq_focus_range_khz = khz;
        if (eng_) status_ = sdrg_engine_set_frequency_focus_range(eng_, khz);
    }
    void setSoundMode(Env *, int32_t mode) {
        cfg_.sound_mode = mode;
        if (eng_) status_ = sdrg_engine_set_sound_mode(eng_, mode);
        if (ssb_) sdrg_ssb_processor_set_sound_mode(ssb_, mode);  // read by the worker per frame (:102)
    }
    void setRefreshFFTMs(Env *, int64_t v) { cfg_.refresh_fft_ms = v; }
    void setRefreshPeakMs(Env *, int64_t v) { cfg_.refresh_peak_ms = v; }
    void setRefreshSignalStrengthMs(Env *, int64_t v) { cfg_.refresh_signal_strength_ms = v; }
    void setPulseConfig(Env *) {}  // legacy parameters ignored, defaults kept (:1156-1160)
    float getAmbientAudioEnergy(Env *) const {  // ssbProcessor.getAmbientEnergy()
        return (mode_ == SsbMode::QUEUED && ssb_) ? sdrg_ssb_processor_get_ambient_energy(ssb_) : audio_.strength;
    }
    float getCurrentAudioRatio(Env *) const {  // ssbProcessor.getCurrentRatio(): always 0 (ssb_processor.h:35)
        return ssb_ ? sdrg_ssb_processor_get_current_ratio(ssb_) : 0.f;
    }

    int32_t lastStatus() const { return status_; }
    const sdrg_config &config() const { return cfg_; }

private:
    struct Cb {
        Obj obj{};
        Mid mid{};
    };
    bool has(int i) const { return cb_[i].obj && cb_[i].mid; }
    void dropCallbacks(Env *env) {
        for (auto &c : cb_) {
            if (c.obj) J::DeleteGlobalRef(env, c.obj);
            c = Cb{};
        }
    }
    // the SSB worker thread's callbacks: attach to the JVM for the call (:701-708, :740-747)
    static void pcmFromWorker(void *u, const int16_t *p, int32_t n) {
        Bridge *b = static_cast<Bridge *>(u);
        if (!b->has(PCM) || n <= 0) return;
        bool attached = false;
        Env *env = J::Attach(b->vm_, &attached);
        if (!env) return;
        J::CallShorts(env, b->cb_[PCM].obj, b->cb_[PCM].mid, p, n);
        J::ClearException(env);
        if (attached) J::Detach(b->vm_);
    }
    static void pulseFromWorker(void *u, float strength, int32_t live_etat) {
        Bridge *b = static_cast<Bridge *>(u);
        if (!b->has(AUDIO_PULSE)) return;
        bool attached = false;
        Env *env = J::Attach(b->vm_, &attached);
        if (!env) return;
        J::CallFI(env, b->cb_[AUDIO_PULSE].obj, b->cb_[AUDIO_PULSE].mid, strength, live_etat);
        J::ClearException(env);
        if (attached) J::Detach(b->vm_);
    }

    sdrg_engine *eng_ = nullptr;
    sdrg_ssb_processor *ssb_ = nullptr;
    SsbMode mode_ = SsbMode::QUEUED;
    Vm vm_{};
    sdrg_config cfg_{};
    Cb cb_[N_CALLBACKS];
    bool reading_ = false;
    int32_t status_ = SDRG_OK;
    std::vector<float> spec_;
    std::vector<int16_t> pcm_;
    sdrg_frame_record rec_{};
    sdrg_pulse_output spectral_{}, audio_{};
};

// The bridge behind one mutex, as the JNI exports use it: the JVM thread (setters, read, stopReading, close), the
// rx thread (frames) and the SSB worker's callbacks (which may call back into the bridge, e.g.
// getAmbientAudioEnergy or setSoundMode from a pcm listener) share it.  Joining the SSB worker never happens
// under the mutex -- a worker blocked in a re-entrant call would never return and the join would deadlock (the
// reference takes no lock around ssbProcessor.stopProcessing, sdr-bridge-java-soapy.cpp:766-793).
template <class J>
class LockedBridge {
public:
    using Br = Bridge<J>;
    using Env = typename J::Env;
    using Obj = typename J::Obj;

    bool applyConfig(Env *env, int64_t cf, int64_t fs, int32_t n, int32_t focus, int32_t gain, int64_t rfft,
                     int64_t rpeak, int64_t rss, int32_t mode) {
        std::lock_guard<std::mutex> lk(mu_);
        return b_.applyConfig(env, cf, fs, n, focus, gain, rfft, rpeak, rss, mode);
    }
    void read(Env *env, const Obj (&cbs)[Br::N_CALLBACKS]) {
        stopWorker();  // read() replaces the callback table the worker reads
        std::lock_guard<std::mutex> lk(mu_);
        b_.read(env, cbs);
    }
    void onFrame(Env *env, const std::complex<float> *buf, uint32_t len, int64_t now_ms) {
        std::lock_guard<std::mutex> lk(mu_);
        b_.onFrame(env, buf, len, now_ms);
    }
    void stopReading(Env *) {
        sdrg_ssb_processor *p;
        {
            std::lock_guard<std::mutex> lk(mu_);
            p = b_.beginStopReading();
        }
        if (p) sdrg_ssb_processor_stop(p);
    }
    void close(Env *env) {
        sdrg_ssb_processor *p;
        {
            std::lock_guard<std::mutex> lk(mu_);
            p = b_.detachSsb();
        }
        if (p) sdrg_ssb_processor_destroy(p);  // joins the worker; its callbacks still see valid global refs
        std::lock_guard<std::mutex> lk(mu_);
        b_.close(env);
    }
    // setters and getters: short, under the lock
    template <class F>
    auto with(F f) -> decltype(f(std::declval<Br &>())) {
        std::lock_guard<std::mutex> lk(mu_);
        return f(b_);
    }
    void setFrequency(Env *e, int64_t v) { with([&](Br &b) { b.setFrequency(e, v); }); }
    void setSampleRate(Env *e, int64_t v) { with([&](Br &b) { b.setSampleRate(e, v); }); }
    void setSamplesPerReading(Env *e, int32_t v) { with([&](Br &b) { b.setSamplesPerReading(e, v); }); }
    void setFrequencyFocusRange(Env *e, int32_t v) { with([&](Br &b) { b.setFrequencyFocusRange(e, v); }); }
    void setSoundMode(Env *e, int32_t v) { with([&](Br &b) { b.setSoundMode(e, v); }); }
    void setRefreshFFTMs(Env *e, int64_t v) { with([&](Br &b) { b.setRefreshFFTMs(e, v); }); }
    void setRefreshPeakMs(Env *e, int64_t v) { with([&](Br &b) { b.setRefreshPeakMs(e, v); }); }
    void setRefreshSignalStrengthMs(Env *e, int64_t v) { with([&](Br &b) { b.setRefreshSignalStrengthMs(e, v); }); }
    void setPulseConfig(Env *e) { with([&](Br &b) { b.setPulseConfig(e); }); }
    float getAmbientAudioEnergy(Env *e) { return with([&](Br &b) { return b.getAmbientAudioEnergy(e); }); }
    float getCurrentAudioRatio(Env *e) { return with([&](Br &b) { return b.getCurrentAudioRatio(e); }); }

private:
    void stopWorker() {
        sdrg_ssb_processor *p;
        {
            std::lock_guard<std::mutex> lk(mu_);
            p = b_.ssbHandle();
        }
        if (p) sdrg_ssb_processor_stop(p);
    }
    std::mutex mu_;
    Br b_;
};

}  // namespace jni
}  // namespace sdrg
