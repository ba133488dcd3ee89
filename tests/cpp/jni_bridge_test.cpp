// jni_bridge_test.cpp — drives sdrg::jni::Bridge (sdr-for-android-lib_amd/jni/sdrg_jni_bridge.hpp) through a
// recording fake of the JNI calls it makes, the way Kotlin's SDRBridge and the reference's rx threads drive
// the JNI exports (applyConfig, read(12 callbacks), frames, setters, stopReading, close), and checks every
// callback's arguments against a second engine driven directly through the C ABI on the same frames:
// the order is soapyCallback's (sdr-bridge-java-soapy.cpp:458-488) then the SSB worker's
// (ssb_processor.cpp:105-113), and every value is bit-identical.  Prints "OK ..." and exits 0 on success.
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "sdrg_jni_bridge.hpp"

namespace {

struct FakeObj {
    int id;
};
struct Call {
    int cb;
    std::string sig;
    std::vector<double> args;   // scalars (float/int/long) as doubles, exactly representable here
    std::vector<float> floats;  // ([F)V payload
    std::vector<int16_t> shorts;
};
struct FakeEnv {
    std::vector<Call> log;
    int global_refs = 0;
};
// the "JVM": the SSB worker thread attaches to it and gets an env of its own (its own call log)
struct FakeVm {
    FakeEnv worker_env;
    int attaches = 0, detaches = 0;
};
FakeVm g_vm;
std::function<void()> g_worker_hook;  // runs inside the SSB worker's pcm callback (re-entrancy test)

struct FakeJni {
    using Env = FakeEnv;
    using Obj = FakeObj *;
    using Mid = const char *;
    using Vm = FakeVm *;
    static Vm VmOf(Env *) { return &g_vm; }
    static Env *Attach(Vm vm, bool *attached) {
        vm->attaches++;  // one worker thread: no lock needed
        *attached = true;
        return &vm->worker_env;
    }
    static void Detach(Vm vm) { vm->detaches++; }
    static Obj NewGlobalRef(Env *e, Obj o) { e->global_refs++; return o; }
    static void DeleteGlobalRef(Env *e, Obj) { e->global_refs--; }
    static Mid MethodOf(Env *, Obj, const char *sig) { return sig; }
    static void ClearException(Env *) {}
    static void push(Env *e, Obj o, Mid m, std::vector<double> a) { e->log.push_back({o->id, m, std::move(a), {}, {}}); }
    static void CallF(Env *e, Obj o, Mid m, float a) { push(e, o, m, {a}); }
    static void CallI(Env *e, Obj o, Mid m, int32_t a) { push(e, o, m, {(double)a}); }
    static void CallJ(Env *e, Obj o, Mid m, int64_t a) { push(e, o, m, {(double)a}); }
    static void CallFF(Env *e, Obj o, Mid m, float a, float b) { push(e, o, m, {a, b}); }
    static void CallFI(Env *e, Obj o, Mid m, float a, int32_t b) { push(e, o, m, {a, (double)b}); }
    static void CallFIJ(Env *e, Obj o, Mid m, float a, int32_t b, int64_t c) { push(e, o, m, {a, (double)b, (double)c}); }
    static void CallFloats(Env *e, Obj o, Mid m, const float *p, int32_t n) {
        e->log.push_back({o->id, m, {}, std::vector<float>(p, p + n), {}});
    }
    static void CallShorts(Env *e, Obj o, Mid m, const int16_t *p, int32_t n) {
        if (e == &g_vm.worker_env && g_worker_hook) g_worker_hook();
        e->log.push_back({o->id, m, {}, {}, std::vector<int16_t>(p, p + n)});
    }
};

using B = sdrg::jni::Bridge<FakeJni>;

int fails = 0;
#define CHECK(c, ...)                                  \
    do {                                               \
        if (!(c)) {                                    \
            std::fprintf(stderr, "FAIL %s: ", #c);     \
            std::fprintf(stderr, __VA_ARGS__);         \
            std::fprintf(stderr, "\n");                \
            if (++fails > 20) return 1;                \
        }                                              \
    } while (0)

bool same_f(double got, float want) { return (float)got == want || (std::isnan(got) && std::isnan(want)); }

}  // namespace

void synth(std::vector<std::complex<float>> &buf, int f, int n, int64_t fs, uint64_t &x) {
    for (int i = 0; i < n; i++) {  // keyed +2 kHz carrier over pseudo-random noise
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        const double t = (double)((int64_t)f * n + i) / fs;
        const double a = (std::fmod(t, 0.45) < 0.08) ? 0.3 : 0.02;
        const double ph = 2 * M_PI * 2000.0 * t;
        buf[i] = {(float)(a * std::cos(ph) + ((double)(x & 0xffff) / 65536.0 - 0.5) * 0.05),
                  (float)(a * std::sin(ph) + ((double)((x >> 16) & 0xffff) / 65536.0 - 0.5) * 0.05)};
    }
}

// QUEUED mode (the reference's SSBProcessor): soapyCallback's 10 callbacks on the frame's thread, pcm + audioPulse
// from the SSB worker thread (attached per call).  Draining the worker after every frame drops nothing, so the
// worker's callbacks must equal the C ABI engine's SSB outputs frame for frame.
int queued_phase() {
    const int n = 4096, frames = 60;
    const int64_t fs = 2000000, cf = 100000000;
    FakeEnv env;
    g_vm = FakeVm{};
    B bridge;
    if (!bridge.applyConfig(&env, cf, fs, n, 5, 10, 50, 200, 30, 1)) return 12;
    FakeObj objs[B::N_CALLBACKS];
    B::Obj cbs[B::N_CALLBACKS];
    for (int i = 0; i < B::N_CALLBACKS; i++) {
        objs[i].id = i;
        cbs[i] = &objs[i];
    }
    bridge.read(&env, cbs);
    sdrg_config c{cf, fs, n, 5, 10, 1, 50, 200, 30};
    sdrg_engine *ref = nullptr;
    if (sdrg_engine_create(&c, 1, 0, &ref)) return 13;
    std::vector<float> spec(n);
    std::vector<int16_t> pcm((size_t)sdrg_engine_pcm_len(ref));
    sdrg_frame_record rec;
    sdrg_pulse_output sp, ap;
    std::vector<std::complex<float>> buf(n);
    uint64_t x = 777;
    for (int f = 0; f < frames; f++) {
        synth(buf, f, n, fs, x);
        env.log.clear();
        g_vm.worker_env.log.clear();
        const int64_t now = 1000 + 2 * f;
        bridge.onFrame(&env, buf.data(), n, now);
        bridge.drainSsb();
        CHECK(bridge.lastStatus() == 0, "queued frame %d status %d", f, bridge.lastStatus());
        if (sdrg_engine_process_host(ref, buf.data(), SDRG_IQ_CF32, SDRG_STAGE_ALL, spec.data(), &rec, pcm.data(), now))
            return 14;
        if (sdrg_engine_get_pulse_outputs(ref, &sp, &ap)) return 15;
        CHECK(env.log.size() == 10, "queued frame %d: %zu frame-thread calls", f, env.log.size());
        CHECK(g_vm.worker_env.log.size() == 2, "queued frame %d: %zu worker calls", f, g_vm.worker_env.log.size());
        if (env.log.size() != 10 || g_vm.worker_env.log.size() != 2) continue;
        CHECK(std::memcmp(env.log[0].floats.data(), spec.data(), 4 * n) == 0, "queued fft payload frame %d", f);
        CHECK(same_f(env.log[9].args[0], rec.best1khz_snr_sigma) && env.log[9].args[1] == sp.live_etat,
              "queued spectralPulse frame %d", f);
        const Call &pc = g_vm.worker_env.log[0], &pu = g_vm.worker_env.log[1];
        CHECK(pc.cb == B::PCM && pc.sig == B::kSignature[B::PCM] && pc.shorts == pcm, "queued pcm frame %d", f);
        CHECK(pu.cb == B::AUDIO_PULSE && same_f(pu.args[0], ap.strength) && pu.args[1] == ap.live_etat,
              "queued audioPulse frame %d", f);
    }
    int64_t enq, drop, proc;
    bridge.ssbCounters(&enq, &drop, &proc);
    CHECK(enq == frames && drop == 0 && proc == frames, "ssb counters %lld %lld %lld", (long long)enq,
          (long long)drop, (long long)proc);
    CHECK(bridge.getAmbientAudioEnergy(&env) == ap.strength, "queued ambient energy");
    CHECK(bridge.getCurrentAudioRatio(&env) == 0.f, "current audio ratio");
    CHECK(g_vm.attaches == g_vm.detaches && g_vm.attaches == 2 * frames, "attach/detach %d %d", g_vm.attaches,
          g_vm.detaches);
    bridge.stopReading(&env);
    bridge.close(&env);
    CHECK(env.global_refs == 0, "queued global refs after close %d", env.global_refs);
    sdrg_engine_destroy(ref);
    return 0;
}

// The JNI exports' lock discipline (sdrg::jni::LockedBridge): a pcm listener on the SSB worker thread that calls
// back into the bridge (getAmbientAudioEnergy, setSoundMode) while the JVM thread runs stopReading or close must
// not deadlock -- the worker is joined outside the bridge's lock.  A watchdog fails the test after 10 s instead of
// hanging.
bool wait_for(const std::atomic<int> &flag, int ms) {
    for (int i = 0; i < ms && !flag.load(); i++) std::this_thread::sleep_for(std::chrono::milliseconds(1));
    return flag.load() != 0;
}

int reentrant_phase() {
    const int n = 4096;
    const int64_t fs = 2000000, cf = 100000000;
    FakeEnv env, env2;
    g_vm = FakeVm{};
    sdrg::jni::LockedBridge<FakeJni> lb;
    if (!lb.applyConfig(&env, cf, fs, n, 5, 10, 50, 200, 30, 1)) return 22;
    FakeObj objs[B::N_CALLBACKS];
    B::Obj cbs[B::N_CALLBACKS];
    for (int i = 0; i < B::N_CALLBACKS; i++) {
        objs[i].id = i;
        cbs[i] = &objs[i];
    }
    std::vector<std::complex<float>> buf(n);
    uint64_t x = 4242;
    std::atomic<int> in_cb{0}, reentered{0};
    g_worker_hook = [&] {
        in_cb.store(1);
        std::this_thread::sleep_for(std::chrono::milliseconds(100));  // the JVM thread's stop starts meanwhile
        (void)lb.getAmbientAudioEnergy(&env2);
        lb.setSoundMode(&env2, 1);
        reentered.fetch_add(1);
    };
    for (int round = 0; round < 2; round++) {  // 0: stopReading, 1: close
        in_cb.store(0);
        lb.read(&env, cbs);
        synth(buf, round, n, fs, x);
        lb.onFrame(&env, buf.data(), n, 1000 + round);
        if (!wait_for(in_cb, 10000)) {
            std::fprintf(stderr, "FAIL reentrant round %d: the worker never called pcm\n", round);
            return 23;
        }
        std::atomic<int> done{0};
        std::thread t([&] {
            if (round == 0)
                lb.stopReading(&env);
            else
                lb.close(&env);
            done.store(1);
        });
        if (!wait_for(done, 10000)) {
            std::fprintf(stderr, "FAIL reentrant round %d: %s deadlocked with a re-entrant pcm callback\n", round,
                         round == 0 ? "stopReading" : "close");
            std::fflush(stderr);
            _exit(9);
        }
        t.join();
        CHECK(reentered.load() == round + 1, "reentrant round %d: %d re-entries", round, reentered.load());
    }
    g_worker_hook = nullptr;
    CHECK(env.global_refs == 0, "reentrant global refs after close %d", env.global_refs);
    return 0;
}

int main() {
    const int n = 4096, frames = 180;
    const int64_t fs = 2000000, cf = 100000000;
    FakeEnv env;
    B bridge;
    bridge.setSsbMode(B::SsbMode::SYNCHRONOUS);
    if (!bridge.applyConfig(&env, cf, fs, n, 5, 10, 50, 200, 30, 1)) {
        std::fprintf(stderr, "applyConfig failed: %s\n", sdrg_last_error());
        return 2;
    }
    FakeObj objs[B::N_CALLBACKS];
    B::Obj cbs[B::N_CALLBACKS];
    for (int i = 0; i < B::N_CALLBACKS; i++) {
        objs[i].id = i;
        cbs[i] = &objs[i];
    }
    bridge.read(&env, cbs);
    CHECK(env.global_refs == B::N_CALLBACKS, "global refs %d", env.global_refs);

    // the same stream through the C ABI
    sdrg_config c{cf, fs, n, 5, 10, 1, 50, 200, 30};
    sdrg_engine *ref = nullptr;
    if (sdrg_engine_create(&c, 1, 0, &ref)) return 3;
    std::vector<float> spec(n);
    std::vector<int16_t> pcm((size_t)sdrg_engine_pcm_len(ref));
    sdrg_frame_record rec;
    sdrg_pulse_output sp, ap;

    std::vector<std::complex<float>> buf(n);
    uint64_t x = 12345;
    for (int f = 0; f < frames; f++) {
        if (f == 60) {  // setFrequency mid-stream, on both
            bridge.setFrequency(&env, cf + 1000);
            sdrg_engine_set_frequency(ref, cf + 1000);
        }
        if (f == 120) {
            bridge.setSoundMode(&env, 2);
            sdrg_engine_set_sound_mode(ref, 2);
        }
        synth(buf, f, n, fs, x);
        env.log.clear();
        const int64_t now = 1000 + 2 * f;
        bridge.onFrame(&env, buf.data(), n, now);
        CHECK(bridge.lastStatus() == 0, "frame %d status %d", f, bridge.lastStatus());
        if (sdrg_engine_process_host(ref, buf.data(), SDRG_IQ_CF32, SDRG_STAGE_ALL, spec.data(), &rec, pcm.data(), now))
            return 4;
        if (sdrg_engine_get_pulse_outputs(ref, &sp, &ap)) return 5;
        // expected sequence
        const int order[] = {B::FFT, B::DETECTION_FLAG, B::MEAN_SNR, B::MEAN_SNR_SIGMA, B::PEAK_FREQUENCY,
                             B::PEAK_ABOVE_NOISE_MEAN, B::MAX_BIN, B::BEST_1KHZ, B::NOISE_LEVEL, B::SPECTRAL_PULSE,
                             B::PCM, B::AUDIO_PULSE};
        CHECK(env.log.size() == 12, "frame %d: %zu calls", f, env.log.size());
        if (env.log.size() != 12) continue;
        for (int k = 0; k < 12; k++) {
            const Call &cl = env.log[k];
            CHECK(cl.cb == order[k], "frame %d call %d is callback %d", f, k, cl.cb);
            CHECK(cl.sig == B::kSignature[cl.cb], "signature %s", cl.sig.c_str());
        }
        CHECK(env.log[0].floats.size() == (size_t)n && std::memcmp(env.log[0].floats.data(), spec.data(), 4 * n) == 0,
              "fft payload frame %d", f);
        CHECK(env.log[1].args[0] == rec.detection_flag, "detection");
        CHECK(same_f(env.log[2].args[0], rec.mean_snr_db), "meanSnr");
        CHECK(same_f(env.log[3].args[0], rec.mean_snr_sigma), "meanSnrSigma");
        CHECK(env.log[4].args[0] == (double)rec.tracking_frequency, "peakFrequency");
        CHECK(same_f(env.log[5].args[0], rec.peak_above_noise_mean_db), "peakAboveNoiseMean");
        CHECK(same_f(env.log[6].args[0], rec.max_bin_snr_db) && same_f(env.log[6].args[1], rec.max_bin_snr_sigma), "maxBin");
        CHECK(same_f(env.log[7].args[0], rec.best1khz_snr_db) && same_f(env.log[7].args[1], rec.best1khz_snr_sigma), "best1kHz");
        CHECK(same_f(env.log[8].args[0], rec.per_bin_mean), "noiseLevel");
        CHECK(same_f(env.log[9].args[0], rec.best1khz_snr_sigma) && env.log[9].args[1] == sp.live_etat &&
                  env.log[9].args[2] == (double)sp.est_freq_hz_rounded, "spectralPulse frame %d", f);
        CHECK(env.log[10].shorts == pcm, "pcm frame %d", f);
        CHECK(same_f(env.log[11].args[0], ap.strength) && env.log[11].args[1] == ap.live_etat, "audioPulse");
    }
    CHECK(bridge.getAmbientAudioEnergy(&env) == ap.strength, "ambient energy");
    bridge.stopReading(&env);
    env.log.clear();
    bridge.onFrame(&env, buf.data(), n, 5000);
    CHECK(env.log.empty(), "callbacks after stopReading");
    bridge.close(&env);
    CHECK(env.global_refs == 0, "global refs after close %d", env.global_refs);
    sdrg_engine_destroy(ref);
    if (fails) return 1;
    const int q = queued_phase();
    if (q) return q;
    const int r = reentrant_phase();
    if (r) return r;
    if (fails) return 1;
    std::printf("OK %d frames, %d callbacks each, spectral live %d, audio live %d; queued SSB worker OK; re-entrant stop/close OK\n", frames, 12,
                sp.live_etat, ap.live_etat);
    return 0;
}
