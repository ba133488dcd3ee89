// pulse_bank.h — host side of the pulse detectors (pulse_bank.cpp): a bank of per-stream detectors of one
// kind with its state in HBM.  The public C ABI (sdrg_pulse_bank_*) and the engine both drive it.
#pragma once

#include <hip/hip_runtime.h>

#include "sdrg_internal.h"

struct sdrg_pulse_bank {
    int kind = SDRG_PULSE_SPECTRAL;
    sdrg_pulse_config cfg{};
    int n_streams = 0;
    int device = 0;
    int cap = 0;                         // ring slots per stream (power of two)
    bool reset_pending = true;           // fresh detectors at the next launch (stream-ordered)
    hipStream_t own_stream = nullptr;
    hipStream_t user_stream = nullptr;   // sdrg_pulse_bank_set_stream
    hipStream_t last_stream = nullptr;   // stream of the last launch (synchronised before a ring regrow)
    hipStream_t detect_stream = nullptr; // engine: the audio detector's stream when it is not the front end's
    sdrg::PulseStreamState *d_state = nullptr;
    float *d_e = nullptr, *d_f = nullptr, *d_rt = nullptr, *d_fh = nullptr;
    int *d_re = nullptr;
    sdrg_pulse_output *d_out = nullptr;  // outputs of the engine-driven / host calls
    float *d_new = nullptr;              // audio: energy frames of one call [NEW_SETS][n_streams][new_slots]
    int *d_new_count = nullptr;          // [NEW_SETS][n_streams]
    // the engine's front end (inside the SSB kernel) and detector (on a stream of its own) of consecutive calls overlap:
    // call k's front end writes set k % NEW_SETS while the detector of call k - 1 reads its own
    static constexpr int NEW_SETS = 3;
    size_t new_slots = 0;
    // host-call staging
    void *d_in = nullptr;
    size_t in_bytes = 0;
};

namespace sdrg {

int32_t fail(int32_t code, const char *fmt, ...);  // engine.cpp: sets sdrg_last_error

int32_t pulse_config_check(int kind, const sdrg_pulse_config *cfg);
int32_t pulse_bank_init(sdrg_pulse_bank *b, int kind, const sdrg_pulse_config *cfg, int n_streams, int device);
void pulse_bank_release(sdrg_pulse_bank *b);
int32_t pulse_bank_configure(sdrg_pulse_bank *b, const sdrg_pulse_config *cfg);
// enqueue one frame per stream on `stream`; out may be the bank's d_out
int32_t pulse_bank_spectral(sdrg_pulse_bank *b, const float *snr_sigma, const float *freq_hz, int stride_bytes,
                            sdrg_pulse_output *out, hipStream_t stream);
int32_t pulse_bank_audio(sdrg_pulse_bank *b, const void *audio, int fmt, int n, int stride, sdrg_pulse_output *out,
                         hipStream_t stream);
// the audio call split for the engine: the SSB kernel runs the front end (af) on the PCM it produces, then
// the detector kernel; n = PCM samples per stream of the call; set = which of the NEW_SETS energy-frame buffers the
// pair uses (the caller keeps a set's detector finished before the front end of a later call writes it again)
int32_t pulse_bank_audio_front(sdrg_pulse_bank *b, int n, AudioFront *af, hipStream_t stream, int set = 0);
int32_t pulse_bank_audio_detect(sdrg_pulse_bank *b, sdrg_pulse_output *out, hipStream_t stream, int set = 0);

}  // namespace sdrg
