// ssb_processor.cpp — SSBProcessor (src/ssb/ssb_processor.h:24-58, ssb_processor.cpp:26-115) over the engine:
// a worker thread fed through a bounded queue that drops its OLDEST frame when full (3 frames, :51-64), so a
// receiver whose SSB consumer falls behind loses SSB frames exactly where the reference does, and the SSB filter
// state runs on over the frames that were processed.  Each frame goes through a one-stream engine's SSB and
// audio-pulse stages (ssb.hip, pulse.hip); then the PCM callback (only when the frame produced samples) and the
// pulse callback (always), as ssbProcessingLoop does (:77-115).
//
// Differences of form, not of behaviour: the queue holds raw frames in any engine format (the reference's is
// CF32 only), the sound mode is this object's (the reference reads the BridgeConfig singleton per frame, :102),
// and the worker's engine is created lazily by the worker thread on the processor's device.
#include <hip/hip_runtime.h>

#include <string.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "pulse_bank.h"
#include "sdrg_internal.h"

using namespace sdrg;

namespace {

struct Item {
    std::vector<uint8_t> bytes;
    int32_t fmt = SDRG_IQ_CF32;
    int32_t n = 0;
    int64_t sample_rate = 0;
};

int32_t bytes_per_sample(int fmt) {
    switch (fmt) {
    case SDRG_IQ_CF32: return 8;
    case SDRG_IQ_CS16: return 4;
    case SDRG_IQ_CS8:
    case SDRG_IQ_CU8: return 2;
    default: return 0;
    }
}

}  // namespace

struct sdrg_ssb_processor {
    int device = 0;
    int queue_max = 3;  // ssb_queue.size() >= 3 -> pop (:58-60)
    std::mutex mu;
    std::condition_variable cv, idle_cv;
    std::deque<Item> q;
    bool busy = false;  // the worker holds a popped frame
    std::thread worker;  // guarded by join_mu
    std::mutex join_mu;  // start / stop / destroy may run on different threads (stopReading vs close)
    // the running worker's id, set by the worker itself before its loop starts: the self-thread checks (a callback
    // that stops, restarts or destroys its own processor) read it without join_mu, which a joiner may hold
    std::atomic<std::thread::id> worker_id{};
    std::atomic<bool> running{false};
    sdrg_ssb_callbacks cbs{};
    std::atomic<int32_t> sound_mode{1};
    std::mutex cfg_mu;  // configMutex_
    bool pending_cfg = false;
    sdrg_pulse_config pending{};
    std::atomic<int64_t> enqueued{0}, dropped{0}, processed{0};
    std::atomic<float> ambient{0.0f};
    std::atomic<int32_t> status{SDRG_OK};
    // worker-owned
    sdrg_engine *eng = nullptr;
    sdrg_config ecfg{};
    std::vector<int16_t> pcm;

    void loop();
    int32_t run_frame(const Item &it);
};

int32_t sdrg_ssb_processor::run_frame(const Item &it) {
    const int32_t mode = sound_mode.load();
    int32_t rc;
    if (!eng) {
        ecfg = sdrg_config{0, it.sample_rate, it.n, 5, 0, mode, 50, 200, 30};
        if ((rc = sdrg_engine_create(&ecfg, 1, device, &eng))) {
            eng = nullptr;
            return rc;
        }
    } else {
        if (ecfg.sample_rate != it.sample_rate && (rc = sdrg_engine_set_sample_rate(eng, it.sample_rate))) return rc;
        if (ecfg.samples_per_reading != it.n && (rc = sdrg_engine_set_samples_per_reading(eng, it.n))) return rc;
        if ((rc = sdrg_engine_set_sound_mode(eng, mode))) return rc;
        ecfg.sample_rate = it.sample_rate;
        ecfg.samples_per_reading = it.n;
        ecfg.sound_mode = mode;
    }
    {  // pulseDetector_ = AudioPulseDetector(pendingConfig_) (:93-99)
        std::lock_guard<std::mutex> lk(cfg_mu);
        if (pending_cfg) {
            if ((rc = sdrg_engine_set_audio_pulse_config(eng, &pending))) return rc;
            pending_cfg = false;
        }
    }
    const int32_t plen = sdrg_engine_pcm_len(eng);
    pcm.resize((size_t)(plen > 0 ? plen : 0));
    if ((rc = sdrg_engine_process_host(eng, it.bytes.data(), it.fmt, SDRG_STAGE_SSB | SDRG_STAGE_AUDIO_PULSE, nullptr,
                                       nullptr, pcm.empty() ? nullptr : pcm.data(), 0)))
        return rc;
    sdrg_pulse_output ap{};
    if ((rc = sdrg_engine_get_pulse_outputs(eng, nullptr, &ap))) return rc;
    ambient.store(ap.strength);
    processed.fetch_add(1);
    if (cbs.pcm && !pcm.empty()) cbs.pcm(cbs.user, pcm.data(), (int32_t)pcm.size());  // :105-107
    if (cbs.pulse) cbs.pulse(cbs.user, ap.strength, ap.live_etat);                    // :109-113
    return SDRG_OK;
}

// ssbProcessingLoop (:77-115)
void sdrg_ssb_processor::loop() {
    while (running.load()) {
        Item it;
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [this] { return !q.empty() || !running.load(); });
            if (!running.load() && q.empty()) break;
            if (q.empty()) continue;
            it = std::move(q.front());
            q.pop_front();
            busy = true;
        }
        const int32_t rc = run_frame(it);
        if (rc) status.store(rc);  // a failed frame is dropped (nothing throws out of the worker)
        {
            std::lock_guard<std::mutex> lk(mu);
            busy = false;
        }
        idle_cv.notify_all();
    }
    {
        std::lock_guard<std::mutex> lk(mu);
        busy = false;
    }
    idle_cv.notify_all();
}

extern "C" {

int32_t sdrg_ssb_processor_create(int32_t device, int32_t queue_max, sdrg_ssb_processor **out) {
    if (!out) return fail(SDRG_E_INVALID, "null out");
    *out = nullptr;
    if (queue_max < 0) return fail(SDRG_E_INVALID, "queue_max must be >= 0");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return fail(SDRG_E_NODEVICE, "no HIP device");
    if (device < 0 || device >= count) return fail(SDRG_E_INVALID, "device %d out of range [0, %d)", device, count);
    sdrg_ssb_processor *p = new sdrg_ssb_processor();
    p->device = device;
    p->queue_max = queue_max > 0 ? queue_max : 3;
    *out = p;
    return SDRG_OK;
}

int32_t sdrg_ssb_processor_stop(sdrg_ssb_processor *p) {
    if (!p) return fail(SDRG_E_INVALID, "null processor");
    {
        std::lock_guard<std::mutex> lk(p->mu);
        p->running.store(false);  // stopProcessing (:40-49)
    }
    p->cv.notify_one();
    // a callback on the worker thread that stops its own processor cannot join itself: the loop ends after it
    if (p->worker_id.load() == std::this_thread::get_id()) return SDRG_OK;
    std::lock_guard<std::mutex> jl(p->join_mu);  // one joiner at a time
    if (p->worker.joinable()) p->worker.join();
    p->worker_id.store(std::thread::id());
    return SDRG_OK;
}

int32_t sdrg_ssb_processor_destroy(sdrg_ssb_processor *p) {
    if (!p) return SDRG_OK;
    // from the worker's own callback the worker is still inside run_frame on this object: refuse (stop() from the
    // callback ends the loop; destroy from another thread afterwards)
    if (p->worker_id.load() == std::this_thread::get_id())
        return fail(SDRG_E_INVALID, "destroy from the worker's own callback");
    sdrg_ssb_processor_stop(p);
    if (p->eng) sdrg_engine_destroy(p->eng);
    delete p;
    return SDRG_OK;
}

int32_t sdrg_ssb_processor_start(sdrg_ssb_processor *p, const sdrg_ssb_callbacks *cbs) {
    if (!p) return fail(SDRG_E_INVALID, "null processor");
    if (p->worker_id.load() == std::this_thread::get_id())
        return p->running.load() ? SDRG_OK : fail(SDRG_E_INVALID, "start from the worker's own callback");
    std::lock_guard<std::mutex> jl(p->join_mu);
    if (p->running.load()) return SDRG_OK;  // "SSB processing already running" (:28-31)
    if (p->worker.joinable()) p->worker.join();  // a loop stopped from its own callback has ended or is ending: reap it
    p->cbs = cbs ? *cbs : sdrg_ssb_callbacks{};
    p->running.store(true);
    p->worker = std::thread([p] {
        p->worker_id.store(std::this_thread::get_id());
        p->loop();
    });
    return SDRG_OK;
}

int32_t sdrg_ssb_processor_enqueue(sdrg_ssb_processor *p, const void *iq, int32_t format, int32_t n,
                                   int64_t sample_rate) {
    if (!p) return fail(SDRG_E_INVALID, "null processor");
    const int bps = bytes_per_sample(format);
    if (!bps) return fail(SDRG_E_INVALID, "unknown iq format %d", format);
    if (n < 1 || n > (1 << 20) || !iq) return fail(SDRG_E_INVALID, "bad frame (n %d)", n);
    if ((uint32_t)sample_rate == 0) return fail(SDRG_E_INVALID, "sample_rate must be > 0");
    if (!p->running.load()) return SDRG_OK;  // ignored when not started (:53)
    Item it;
    it.bytes.assign(static_cast<const uint8_t *>(iq), static_cast<const uint8_t *>(iq) + (size_t)n * bps);
    it.fmt = format;
    it.n = n;
    it.sample_rate = sample_rate;
    {
        std::lock_guard<std::mutex> lk(p->mu);
        while ((int)p->q.size() >= p->queue_max) {  // drop the oldest (:58-60)
            p->q.pop_front();
            p->dropped.fetch_add(1);
        }
        p->q.push_back(std::move(it));
        p->enqueued.fetch_add(1);
    }
    p->cv.notify_one();
    return SDRG_OK;
}

int32_t sdrg_ssb_processor_set_sound_mode(sdrg_ssb_processor *p, int32_t mode) {
    if (!p) return fail(SDRG_E_INVALID, "null processor");
    p->sound_mode.store(mode);
    return SDRG_OK;
}

int32_t sdrg_ssb_processor_set_pulse_config(sdrg_ssb_processor *p, const sdrg_pulse_config *cfg) {
    if (!p) return fail(SDRG_E_INVALID, "null processor");
    int32_t rc = pulse_config_check(SDRG_PULSE_AUDIO, cfg);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(p->cfg_mu);
    p->pending = *cfg;
    p->pending_cfg = true;
    return SDRG_OK;
}

float sdrg_ssb_processor_get_ambient_energy(const sdrg_ssb_processor *p) { return p ? p->ambient.load() : 0.0f; }

float sdrg_ssb_processor_get_current_ratio(const sdrg_ssb_processor *) { return 0.0f; }

int32_t sdrg_ssb_processor_drain(sdrg_ssb_processor *p) {
    if (!p) return fail(SDRG_E_INVALID, "null processor");
    std::unique_lock<std::mutex> lk(p->mu);
    p->idle_cv.wait(lk, [p] { return (p->q.empty() || !p->running.load()) && !p->busy; });
    return SDRG_OK;
}

int32_t sdrg_ssb_processor_counters(const sdrg_ssb_processor *p, int64_t *enqueued, int64_t *dropped,
                                    int64_t *processed, int32_t *last_status) {
    if (!p) return fail(SDRG_E_INVALID, "null processor");
    if (enqueued) *enqueued = p->enqueued.load();
    if (dropped) *dropped = p->dropped.load();
    if (processed) *processed = p->processed.load();
    if (last_status) *last_status = p->status.load();
    return SDRG_OK;
}

}  // extern "C"
