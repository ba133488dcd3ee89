// sdrg_jni.cpp — the JNI exports of Kotlin's SDRBridge object (java/fr/intuite/sdr/bridge/SDRBridge.kt) over
// sdrg::jni::Bridge.  Built only in the Android bridge's CMake target, next to libsdrg.so and the NDK's
// <jni.h> (this image has no JDK/NDK, so it is compiled here only against the test fake, through
// sdrg_jni_bridge.hpp).  The SoapySDR device side (initDongle, the rx threads) stays
// in the bridge: its rx_process_thread hands each exact-N chunk to sdrg_jni_on_frame() instead of
// soapyCallback().
#include <jni.h>

#include <chrono>

#include "sdrg_jni_bridge.hpp"

namespace {

struct RealJni {
    using Env = JNIEnv;
    using Obj = jobject;
    using Mid = jmethodID;
    using Vm = JavaVM *;
    static Vm VmOf(Env *e) {
        JavaVM *vm = nullptr;
        return e->GetJavaVM(&vm) == JNI_OK ? vm : nullptr;
    }
    // the SSB worker thread's JNIEnv (sdr-bridge-java-soapy.cpp:701-708)
    static Env *Attach(Vm vm, bool *attached) {
        *attached = false;
        if (!vm) return nullptr;
        JNIEnv *env = nullptr;
        const jint r = vm->GetEnv(reinterpret_cast<void **>(&env), JNI_VERSION_1_6);
        if (r == JNI_OK) return env;
        if (r != JNI_EDETACHED || vm->AttachCurrentThread(&env, nullptr) != JNI_OK) return nullptr;
        *attached = true;
        return env;
    }
    static void Detach(Vm vm) { vm->DetachCurrentThread(); }
    static Obj NewGlobalRef(Env *e, Obj o) { return e->NewGlobalRef(o); }
    static void DeleteGlobalRef(Env *e, Obj o) { e->DeleteGlobalRef(o); }
    static Mid MethodOf(Env *e, Obj o, const char *sig) {
        jclass c = e->GetObjectClass(o);
        Mid m = e->GetMethodID(c, "invoke", sig);
        e->DeleteLocalRef(c);
        return m;
    }
    static void ClearException(Env *e) {
        if (e->ExceptionCheck()) e->ExceptionClear();
    }
    static void CallF(Env *e, Obj o, Mid m, float a) { e->CallVoidMethod(o, m, (jfloat)a); }
    static void CallI(Env *e, Obj o, Mid m, int32_t a) { e->CallVoidMethod(o, m, (jint)a); }
    static void CallJ(Env *e, Obj o, Mid m, int64_t a) { e->CallVoidMethod(o, m, (jlong)a); }
    static void CallFF(Env *e, Obj o, Mid m, float a, float b) { e->CallVoidMethod(o, m, (jfloat)a, (jfloat)b); }
    static void CallFI(Env *e, Obj o, Mid m, float a, int32_t b) { e->CallVoidMethod(o, m, (jfloat)a, (jint)b); }
    static void CallFIJ(Env *e, Obj o, Mid m, float a, int32_t b, int64_t c) {
        e->CallVoidMethod(o, m, (jfloat)a, (jint)b, (jlong)c);
    }
    static void CallFloats(Env *e, Obj o, Mid m, const float *p, int32_t n) {  // fresh array per frame (:458-466)
        jfloatArray a = e->NewFloatArray(n);
        if (!a) return;
        e->SetFloatArrayRegion(a, 0, n, p);
        e->CallVoidMethod(o, m, a);
        e->DeleteLocalRef(a);
    }
    static void CallShorts(Env *e, Obj o, Mid m, const int16_t *p, int32_t n) {
        jshortArray a = e->NewShortArray(n);
        if (!a) return;
        e->SetShortArrayRegion(a, 0, n, p);
        e->CallVoidMethod(o, m, a);
        e->DeleteLocalRef(a);
    }
};

// the JVM thread (setters), the rx thread (frames) and the SSB worker's callbacks share the bridge; LockedBridge
// serialises them and joins the worker outside its lock
sdrg::jni::LockedBridge<RealJni> g_bridge;

int64_t now_ms() {
    return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

}  // namespace

// Called by the bridge's rx_process_thread for each exact-N chunk (replaces soapyCallback).
extern "C" void sdrg_jni_on_frame(JNIEnv *env, const std::complex<float> *buf, uint32_t len) {
    g_bridge.onFrame(env, buf, len, now_ms());
}

extern "C" JNIEXPORT jboolean JNICALL Java_fr_intuite_sdr_bridge_SDRBridge_applyConfig(
    JNIEnv *env, jobject, jlong cf, jlong fs, jint n, jint focus, jint gain, jlong rfft, jlong rpeak, jlong rss,
    jint mode) {
    return g_bridge.applyConfig(env, cf, fs, n, focus, gain, rfft, rpeak, rss, mode) ? JNI_TRUE : JNI_FALSE;
}

extern "C" JNIEXPORT void JNICALL Java_fr_intuite_sdr_bridge_SDRBridge_read(
    JNIEnv *env, jobject, jobject fft, jobject detectionFlag, jobject meanSnr, jobject meanSnrSigma,
    jobject peakFrequency, jobject pcm, jobject audioPulse, jobject peakAboveNoiseMean, jobject maxBin,
    jobject best1kHz, jobject spectralPulse, jobject noiseLevel) {
    const jobject cbs[] = {fft, detectionFlag, meanSnr, meanSnrSigma, peakFrequency, pcm, audioPulse,
                           peakAboveNoiseMean, maxBin, best1kHz, spectralPulse, noiseLevel};
    g_bridge.read(env, cbs);
}

extern "C" JNIEXPORT void JNICALL Java_fr_intuite_sdr_bridge_SDRBridge_stopReading(JNIEnv *env, jobject) {
    g_bridge.stopReading(env);
}

extern "C" JNIEXPORT void JNICALL Java_fr_intuite_sdr_bridge_SDRBridge_close(JNIEnv *env, jobject) {
    g_bridge.close(env);
}

#define SDRG_JNI_SETTER(NAME, JT, CALL)                                                                    \
    extern "C" JNIEXPORT void JNICALL Java_fr_intuite_sdr_bridge_SDRBridge_##NAME(JNIEnv *env, jobject, JT v) { \
        g_bridge.CALL(env, v);                                                                             \
    }
SDRG_JNI_SETTER(setFrequency, jlong, setFrequency)
SDRG_JNI_SETTER(setSampleRate, jlong, setSampleRate)
SDRG_JNI_SETTER(setSamplesPerReading, jint, setSamplesPerReading)
SDRG_JNI_SETTER(setFrequencyFocusRange, jint, setFrequencyFocusRange)
SDRG_JNI_SETTER(setSoundMode, jint, setSoundMode)
SDRG_JNI_SETTER(setRefreshFFTMs, jlong, setRefreshFFTMs)
SDRG_JNI_SETTER(setRefreshPeakMs, jlong, setRefreshPeakMs)
SDRG_JNI_SETTER(setRefreshSignalStrengthMs, jlong, setRefreshSignalStrengthMs)
#undef SDRG_JNI_SETTER

extern "C" JNIEXPORT void JNICALL Java_fr_intuite_sdr_bridge_SDRBridge_setPulseConfig(
    JNIEnv *env, jobject, jfloat, jfloat, jfloat, jfloat, jfloat, jfloat, jfloat, jfloat, jfloat) {
    g_bridge.setPulseConfig(env);
}

extern "C" JNIEXPORT jfloat JNICALL Java_fr_intuite_sdr_bridge_SDRBridge_getAmbientAudioEnergy(JNIEnv *env, jobject) {
    return g_bridge.getAmbientAudioEnergy(env);
}

// getCurrentAudioRatio (sdr-bridge-java-soapy.cpp:1168-1171): ssbProcessor.getCurrentRatio(), always 0
extern "C" JNIEXPORT jfloat JNICALL Java_fr_intuite_sdr_bridge_SDRBridge_getCurrentAudioRatio(JNIEnv *env, jobject) {
    return g_bridge.getCurrentAudioRatio(env);
}
