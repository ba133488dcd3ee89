// sdrg_internal.h — kernel launchers shared by the engine (host C++) and the HIP translation units.
// Not part of the public ABI (include/sdrg.h is).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sdrg_types.h"

#include <stdlib.h>

// Lab knobs (tools/: role maps, priorities, CU splits, stamps ...) are read from the environment only in lab
// builds (-DSDRG_LAB=1, tools/build_variant.sh); the product library (make) ignores them, so a stray variable in
// a deployed process cannot change its results or its schedule.
#ifndef SDRG_LAB
#define SDRG_LAB 0
#endif
static inline const char *lab_getenv(const char *name) { return SDRG_LAB ? getenv(name) : nullptr; }

namespace sdrg {

// Raise a kernel's dynamic-LDS limit to `bytes` on the CURRENT device, once per (kernel, device): the
// attribute is per device, and engines on several devices or threads may launch the same kernel
// concurrently (engine.cpp; mutex-protected).
hipError_t ensure_dynamic_lds(const void *kernel, int bytes);

// Makes `device` current for the scope of an entry point and restores the caller's current device on
// exit, so the C ABI never leaves the calling thread on another device (engine.cpp, pulse_bank.cpp).
class DeviceScope {
public:
    explicit DeviceScope(int device) {
        if (hipGetDevice(&prev_) != hipSuccess) prev_ = -1;
        err_ = (prev_ == device) ? hipSuccess : hipSetDevice(device);
        changed_ = err_ == hipSuccess && prev_ != device;
    }
    ~DeviceScope() {
        if (changed_ && prev_ >= 0) (void)hipSetDevice(prev_);
    }
    DeviceScope(const DeviceScope &) = delete;
    DeviceScope &operator=(const DeviceScope &) = delete;
    hipError_t error() const { return err_; }

private:
    int prev_ = -1;
    bool changed_ = false;
    hipError_t err_ = hipSuccess;
};

// ------------------------------------------------------------------------------------------------
// Launchers (defined in the .hip translation units).  All are asynchronous on `stream`.
// ------------------------------------------------------------------------------------------------
// Spectrum kernels, every N in [1, 2^20]: powers of two 64 .. 16384 one LDS-resident workgroup per frame,
// 32768/65536 two-kernel four-step in waves of spectrum_wave_frames(n) frames, 128 MiB of complex intermediate
// (`scratch`, spectrum_scratch_floats() floats) that stays in the 256 MiB Infinity Cache (measured at 65536:
// 64 / 128 / 256 / 512 frames per wave 0.418 / 0.356 / 0.318 / 0.393 ms per 1024 frames); every other N through
// fftany.hip (mixed radix, four-step, Bluestein).
#ifndef SDRG_SPECTRUM_WAVE_FRAMES  // lab override of the 65536-point wave (tools/build_variant.sh); 0: 128 MiB
#define SDRG_SPECTRUM_WAVE_FRAMES 0
#endif
constexpr size_t SPECTRUM_WAVE_BYTES = (size_t)128 << 20;
inline int spectrum_wave_frames(int n) {
    if (SDRG_SPECTRUM_WAVE_FRAMES > 0) return SDRG_SPECTRUM_WAVE_FRAMES * (65536 / n);
    return (int)(SPECTRUM_WAVE_BYTES / ((size_t)n * 8));
}
bool spectrum_supported(int n);
size_t spectrum_scratch_floats(int n, int n_frames);
// Twiddle buffer the spectrum kernels read (floats) and its contents for frame size n.
size_t spectrum_twiddle_floats(int n);
void spectrum_fill_twiddles(int n, float *out);
// twiddles: exp(-2 pi i m / N), m in [0, N), float2, computed in double on the host.
// beside_ssb: the previous call's SSB pipeline is expected to hold the CUs (pipelined calls); the persistent
// N = 16384 kernel then launches one workgroup per CU, the one that co-resides with it (measured +2-3 % per
// step over two), instead of two per CU for the chip alone.
// n_cus: CUs the stream may use (0 = the device's; a CU-masked stream passes its share) for persistent grids.
// beside_wide_stats: the call's statistics take the wide kernel (its workgroups share the CUs with the next call's
// FFT): N = 32768 / 65536 then launch one tile per workgroup instead of the persistent four-step kernels.
hipError_t launch_spectrum(const void *iq, int fmt, int n, int n_frames, const float *twiddles,
                           float *spectra, float *scratch, hipStream_t stream, bool beside_ssb = false, int n_cus = 0,
                           bool beside_wide_stats = false);
// true when launch_stats runs this geometry with the wide kernel (stats.hip)
bool stats_uses_wide(const StatsGeometry &geo);

// gpool: [n_frames][stats_global_pool_floats / n_frames] device scratch for the pooled-bin median when the
// pool exceeds what the kernel keeps in LDS (stats_global_pool_floats > 0; wide focus windows at N > 65536)
size_t stats_global_pool_floats(const StatsGeometry &geo, int n_frames);
hipError_t launch_stats(const float *spectra, int n_frames, const StatsGeometry &geo, int64_t now_ms,
                        StatsState *state, sdrg_frame_record *records, float *gpool, hipStream_t stream);

// SSB chain.  The pipelined kernel needs no scratch; the lane-per-stream reference kernels (used for
// sample rates below ~0.9 MHz, or when SDRG_SSB_REFERENCE_KERNELS=1) need
// scratch: [n_frames][samp_count + pcm_len] floats.  taps: [n_taps] device floats.
bool ssb_force_reference_kernels();
void ssb_report_stamps();  // diagnostic (SDRG_PIPE_STAMPS=1)
// chunk_table: per chunk of ssb_pipe_chunk() samples {first, last output overlapping it, first, last output
// completed in it} (host-computed, see engine.cpp); may be null (reference kernels).
int ssb_pipe_chunk(void);
// audio (nullable): run the audio pulse detector's front end on the PCM as it is produced
// stop: an event the pipeline kernel may complete itself (*stop_recorded = true); otherwise the caller records it
hipError_t launch_ssb(const void *iq, int fmt, int n_frames, const SsbParams &p, const float *taps,
                      const int *chunk_table, SsbStreamState *state, float *scratch, int16_t *pcm,
                      const AudioFront *audio, hipStream_t stream, hipEvent_t stop = nullptr,
                      bool *stop_recorded = nullptr);

// Pulse detectors (pulse.hip): one wavefront per stream.  Rings are [n_streams][cap] (cap = cap_mask + 1),
// fh [n_streams][2][PULSE_FH_SLOTS].
hipError_t launch_pulse_reset(PulseStreamState *states, int n_streams, float t_target_init, hipStream_t stream);
hipError_t launch_spectral_pulse(const PulseParams &p, int n_streams, PulseStreamState *states, float *ebuf,
                                 float *fbuf, float *roi_t, int *roi_etat, float *fh, const float *snr_sigma,
                                 const float *freq_hz, int stride_bytes, sdrg_pulse_output *out, hipStream_t stream);
// audio: the front end (lane per stream; also fused into the SSB kernels, see launch_ssb) writes each call's
// energy values to a.new_e [n_streams][a.max_new] (a.max_new >= n_samples / frame_samples + 1) and counts;
// the detector (wave per stream) consumes them.
hipError_t launch_audio_front(const AudioFront &a, const void *audio, int fmt, int n_samples, int stride, int n_streams,
                              hipStream_t stream);
hipError_t launch_audio_detect(const PulseParams &p, int n_streams, PulseStreamState *states, float *ebuf, float *roi_t,
                               int *roi_etat, const float *new_e, int max_new, const int *new_count,
                               sdrg_pulse_output *out, hipStream_t stream);

// Sets the thread's sdrg_last_error message and returns code (engine.cpp).
int32_t fail(int32_t code, const char *fmt, ...);

// Multi-GPU (dist.cpp, gather.hip).  One gather per item, all in one RCCL group on `stream`: every rank sends
// items[i].bytes from items[i].send; the root receives world x bytes at items[i].recv in rank order.
struct GatherItem {
    const void *send;
    void *recv;
    size_t bytes;
};
int32_t dist_gather(sdrg_dist *d, const GatherItem *items, int n_items, int root, hipStream_t stream);
int dist_device(const sdrg_dist *d);
int dist_world(const sdrg_dist *d);
int dist_rank(const sdrg_dist *d);
// out[s][j] = spectra[s][lo + j], j < nb: each stream's focus-window slice, contiguous for the gather
// gather.hip: the read + write GB/s of a float4 streaming copy of `bytes` (reps timed launches) on the current device
hipError_t measure_stream_copy(size_t bytes, int reps, double *gbs);
hipError_t launch_focus_pack(const float *spectra, int n_streams, int n, int lo, int nb, float *out, hipStream_t stream);

}  // namespace sdrg
