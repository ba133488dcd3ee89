// jni.h — TEST INFRASTRUCTURE ONLY (tests/test_jni_exports.py).  A minimal header shaped after the JNI
// specification's C++ interface (the types, constants and the JNIEnv / JavaVM members sdrg_jni.cpp calls), so that
// jni/sdrg_jni.cpp compiles here, where the image has neither a JDK nor the Android NDK.  It pins nothing about a
// real JVM: the members are declared, never defined, and the object file is only inspected (nm), never linked.
#pragma once
#include <stdarg.h>
#include <stdint.h>

typedef uint8_t jboolean;
typedef int8_t jbyte;
typedef uint16_t jchar;
typedef int16_t jshort;
typedef int32_t jint;
typedef int64_t jlong;
typedef float jfloat;
typedef double jdouble;
typedef jint jsize;

class _jobject {};
class _jclass : public _jobject {};
class _jarray : public _jobject {};
class _jfloatArray : public _jarray {};
class _jshortArray : public _jarray {};
typedef _jobject *jobject;
typedef _jclass *jclass;
typedef _jfloatArray *jfloatArray;
typedef _jshortArray *jshortArray;
struct _jmethodID;
typedef _jmethodID *jmethodID;

#define JNI_FALSE 0
#define JNI_TRUE 1
#define JNI_OK 0
#define JNI_EDETACHED (-2)
#define JNI_VERSION_1_6 0x00010006
#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL

struct _JavaVM;
typedef _JavaVM JavaVM;

struct _JNIEnv {
    jint GetJavaVM(JavaVM **vm);
    jclass GetObjectClass(jobject obj);
    jmethodID GetMethodID(jclass clazz, const char *name, const char *sig);
    void DeleteLocalRef(jobject obj);
    jobject NewGlobalRef(jobject obj);
    void DeleteGlobalRef(jobject obj);
    jboolean ExceptionCheck();
    void ExceptionClear();
    void CallVoidMethod(jobject obj, jmethodID methodID, ...);
    jfloatArray NewFloatArray(jsize length);
    void SetFloatArrayRegion(jfloatArray array, jsize start, jsize len, const jfloat *buf);
    jshortArray NewShortArray(jsize length);
    void SetShortArrayRegion(jshortArray array, jsize start, jsize len, const jshort *buf);
};
typedef _JNIEnv JNIEnv;

struct _JavaVM {
    jint GetEnv(void **env, jint version);
    jint AttachCurrentThread(JNIEnv **p_env, void *thr_args);
    jint DetachCurrentThread();
};
