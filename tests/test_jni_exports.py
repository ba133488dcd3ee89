"""The JNI exports (sdr-for-android-lib_amd/jni/sdrg_jni.cpp) compile, and they are exactly the DSP-side subset of the
reference's SDRBridge natives, with the JNI types of their Kotlin declarations.

The image has no JDK / NDK, so the file is compiled against tests/cpp/jni_spec/jni.h, a minimal header shaped after
the JNI specification (test infrastructure: it pins nothing about a real JVM).  Two checks:
* `nm` of the object file: the defined Java_fr_intuite_sdr_bridge_SDRBridge_* symbols equal EXPORTS below;
* a second translation unit declares every export with the prototype its Kotlin `external fun` maps to (Long ->
  jlong, Int -> jint, Float -> jfloat, Boolean -> jboolean, a lambda -> jobject) BEFORE including sdrg_jni.cpp: two
  extern "C" declarations of one name with different types do not compile, so a wrong parameter list fails here.

EXPORTS is the reference's list (/root/reference/src/sdr-bridge-java-soapy.cpp:625, 766, 796, 878-1071, 1073, 1143,
1163, 1168; Kotlin declarations java/fr/intuite/sdr/bridge/SDRBridge.kt:77-213) minus the SoapySDR device side the
bridge keeps (initDongle, getDriver, setGain, getGain, getTunerGains, getFrequency, getFrequencyRange, getSampleRate,
getSampleRatesList).
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JNI_DIR = os.path.join(ROOT, "sdr-for-android-lib_amd", "jni")
SPEC = os.path.join(ROOT, "tests", "cpp", "jni_spec")
PREFIX = "Java_fr_intuite_sdr_bridge_SDRBridge_"

# name: (JNI return type, parameter JNI types after (JNIEnv *, jobject)) from the Kotlin declarations
EXPORTS = {
    "setPulseConfig": ("void", ["jfloat"] * 9),                                          # SDRBridge.kt:77-87
    "applyConfig": ("jboolean", ["jlong", "jlong", "jint", "jint", "jint", "jlong", "jlong", "jlong", "jint"]),  # :130-139
    "read": ("void", ["jobject"] * 12),                                                  # :141-154
    "stopReading": ("void", []),                                                         # :156
    "close": ("void", []),                                                               # :158
    "setFrequency": ("void", ["jlong"]),                                                 # :163
    "setFrequencyFocusRange": ("void", ["jint"]),                                        # :164
    "setSampleRate": ("void", ["jlong"]),                                                # :185
    "setSamplesPerReading": ("void", ["jint"]),                                          # :186
    "setRefreshFFTMs": ("void", ["jlong"]),                                              # :199
    "setRefreshPeakMs": ("void", ["jlong"]),                                             # :200
    "setRefreshSignalStrengthMs": ("void", ["jlong"]),                                   # :201
    "setSoundMode": ("void", ["jint"]),                                                  # :209
    "getAmbientAudioEnergy": ("jfloat", []),                                             # :211
    "getCurrentAudioRatio": ("jfloat", []),                                              # :213
}

CXX = shutil.which("g++")


def _compile(src, obj):
    cmd = [CXX, "-std=c++17", "-fPIC", "-O1", "-Wall", "-Werror", "-c", src, "-o", obj, f"-I{SPEC}", f"-I{JNI_DIR}",
           f"-I{os.path.join(ROOT, 'include')}"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]


@pytest.mark.skipif(CXX is None, reason="no g++")
def test_jni_exports_compile_and_match(tmp_path):
    obj = str(tmp_path / "sdrg_jni.o")
    _compile(os.path.join(JNI_DIR, "sdrg_jni.cpp"), obj)
    nm = subprocess.run(["nm", "-g", "--defined-only", obj], capture_output=True, text=True, check=True).stdout
    got = {l.split()[-1][len(PREFIX):] for l in nm.splitlines() if l.split() and l.split()[-1].startswith(PREFIX)}
    assert got == set(EXPORTS), (sorted(got - set(EXPORTS)), sorted(set(EXPORTS) - got))


@pytest.mark.skipif(CXX is None, reason="no g++")
def test_jni_export_signatures_follow_kotlin(tmp_path):
    src = tmp_path / "sig_check.cpp"
    lines = ["#include <jni.h>"]
    for name, (ret, params) in EXPORTS.items():
        args = ", ".join(["JNIEnv *", "jobject"] + params)
        lines.append(f'extern "C" JNIEXPORT {ret} JNICALL {PREFIX}{name}({args});')
    lines.append(f'#include "{os.path.join(JNI_DIR, "sdrg_jni.cpp")}"')
    src.write_text("\n".join(lines) + "\n")
    _compile(str(src), str(tmp_path / "sig_check.o"))


@pytest.mark.skipif(CXX is None, reason="no g++")
def test_signature_check_catches_a_wrong_type(tmp_path):
    """the prototype trick is live: a deliberately wrong parameter type must fail to compile"""
    src = tmp_path / "sig_bad.cpp"
    src.write_text("#include <jni.h>\n"
                   f'extern "C" JNIEXPORT void JNICALL {PREFIX}setFrequency(JNIEnv *, jobject, jint);\n'
                   f'#include "{os.path.join(JNI_DIR, "sdrg_jni.cpp")}"\n')
    r = subprocess.run([CXX, "-std=c++17", "-c", str(src), "-o", str(tmp_path / "bad.o"), f"-I{SPEC}", f"-I{JNI_DIR}",
                        f"-I{os.path.join(ROOT, 'include')}"], capture_output=True, text=True)
    assert r.returncode != 0 and "conflicting" in r.stderr
