/*
 * sdrg.h — C ABI of the MI355X (gfx950) IQ-stream DSP engine.
 *
 * This is the drop-in boundary for the reference's per-frame hot path
 * (alexandreGellibert/SDR-for-Android-lib, paths relative to the reference root):
 *
 *   FFTProcessor::configure / process / get*      src/dsp/fft_process.h:29-55, fft_process.cpp:20-379
 *   processSSB_opt(iq, fs, upper, pcm, pulse, mode) src/ssb/ssb_demod_opt.h:64-65, ssb_demod_opt.cpp:221-296
 *   SSBProcessor (queue + worker)                  src/ssb/ssb_processor.h:24-58
 *   JNI applyConfig / read / set*                  src/sdr-bridge-java-soapy.cpp:625-764, 878-1141
 *   SDRConfig fields                               java/fr/intuite/sdr/bridge/SDRBridge.kt:23-37
 *
 * The reference runs one receiver ("stream") per process and processes one frame of
 * samplesPerReading complex samples per call.  The engine generalises that to B independent
 * streams processed one frame each per call ("B streams x 1 frame per launch"): every piece of
 * per-stream state the reference keeps in FFTProcessor members or in processSSB_opt's
 * function statics is kept per stream in HBM, so stream s of a batch behaves exactly like a
 * reference process that was fed stream s's frames in order.
 *
 * Conventions: plain pointers and sizes, no exceptions across the boundary, every entry point
 * returns an sdrg_status (0 = OK).  A handle is not safe for concurrent calls from several
 * threads; configuration changes are applied at the next process call (frame boundary), which
 * replaces the reference's racy configure()-while-process() pattern (sdr-bridge-java-soapy.cpp:878-913).
 */
#ifndef SDRG_H
#define SDRG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SDRG_ABI_VERSION 1

/* Status codes.  The reference's JNI layer reports failure as false/nullptr/0 plus a log line
 * (e.g. applyConfig returns false when a device call throws, sdr-bridge-java-soapy.cpp:1115-1118). */
typedef enum sdrg_status {
    SDRG_OK = 0,
    SDRG_E_INVALID = -1,      /* bad argument (null pointer, non-positive size, ...) */
    SDRG_E_UNSUPPORTED = -2,  /* e.g. a frame size outside [1, 2^20] */
    SDRG_E_NOMEM = -3,        /* device allocation failed */
    SDRG_E_HIP = -4,          /* a HIP runtime call failed (message via sdrg_last_error) */
    SDRG_E_NODEVICE = -5      /* no gfx950 device / HIP runtime not usable */
} sdrg_status;

/* Raw IQ sample formats.  The reference stream is always CF32 (sdr-bridge-java-soapy.cpp:263);
 * the device drivers convert their native CU8 / CS8 / CS16 to CF32 before the hot path.  The
 * engine fuses that conversion into its kernels with the convention
 *   CS8: v/128      CU8: (v - 127.4f) * (1/128)  (the in-tree convertIQ, ssb_demod_opt.cpp:33-44)
 *   CS16: v/32768   CF32: as is.  Samples are interleaved I,Q. */
typedef enum sdrg_iq_format {
    SDRG_IQ_CF32 = 0,
    SDRG_IQ_CS8 = 1,
    SDRG_IQ_CU8 = 2,
    SDRG_IQ_CS16 = 3,
    SDRG_IQ_CS12 = 4   /* packed 12-bit (3 bytes per complex sample): sdrg_ingest input only, repacked to CS16 */
} sdrg_iq_format;

/* Which stages a process call runs (bitmask). */
enum {
    SDRG_STAGE_SPECTRUM = 1,  /* FFT -> |X|^2 -> fftshift (fft_process.cpp:42-97) */
    SDRG_STAGE_STATS = 2,     /* evaluateSignalStrength (fft_process.cpp:122-379); needs SPECTRUM */
    SDRG_STAGE_SSB = 4,       /* processSSB_opt (ssb_demod_opt.cpp:221-296) */
    SDRG_STAGE_HOT_PATH = 7,  /* the three above: the accelerated per-frame DSP path */
    SDRG_STAGE_SPECTRAL_PULSE = 8,  /* SpectralPulseDetector::process(best1kHzSnrSigma, best1kHzCenterFreqHz)
                                       (sdr-bridge-java-soapy.cpp:477-488); needs STATS */
    SDRG_STAGE_AUDIO_PULSE = 16,    /* AudioPulseDetector::process(pcm) (ssb_processor.cpp:109-113); needs SSB */
    SDRG_STAGE_ALL = 31             /* everything soapyCallback + the SSB worker do per frame */
};

/* Mirror of Kotlin SDRConfig (SDRBridge.kt:23-37) / the 9 JNI applyConfig arguments
 * (sdr-bridge-java-soapy.cpp:1073-1085).  gain and refresh_* are carried for API parity only:
 * gain is a device setting and the refresh periods are stored but never read by the reference. */
typedef struct sdrg_config {
    int64_t center_frequency;          /* Hz; the reference stores it as uint32 (bridge-config.h:18) */
    int64_t sample_rate;               /* Hz; uint32 in the reference */
    int32_t samples_per_reading;       /* frame size N: any N in [1, 2^20] (fftwf_plan_dft_1d plans any N,
                                          fft_process.cpp:77-79; SDRBridge.kt:25 recommends multiples of 512) */
    int32_t freq_focus_range_khz;      /* focus half-width X in kHz */
    int32_t gain;
    int32_t sound_mode;                /* 0,1,2 (SDRBridge.kt:35-36); other values keep the last mode */
    int64_t refresh_fft_ms;
    int64_t refresh_peak_ms;
    int64_t refresh_signal_strength_ms;
} sdrg_config;

/* Per-frame, per-stream outputs: exactly what soapyCallback reads through the FFTProcessor getters
 * (sdr-bridge-java-soapy.cpp:446-455, fft_process.h:38-55), plus a few diagnostics for parity. */
typedef struct sdrg_frame_record {
    int64_t tracking_frequency;        /* getTrackingFrequency(): lround-ish of the float latch */
    float mean_snr_db;                 /* getMeanSnrDb */
    float mean_snr_sigma;              /* getMeanSnrSigma */
    float peak_above_noise_mean_db;    /* getPeakAboveNoiseMeanDb */
    float max_bin_snr_db;              /* getMaxBinSnrDb */
    float max_bin_snr_sigma;           /* getMaxBinSnrSigma */
    float best1khz_snr_db;             /* getBest1kHzSnrDb */
    float best1khz_snr_sigma;          /* getBest1kHzSnrSigma */
    float best1khz_center_freq_hz;     /* getBest1kHzCenterFreqHz */
    float per_bin_mean;                /* getPerBinMean (noiseLevel callback) */
    int32_t detection_flag;            /* getDetectionFlag: 0 or 3 */
    /* diagnostics (not reference getters) */
    int32_t peak_bin;                  /* focusLo + peakBinInFocus of this frame (-1 if no focus window) */
    float abs_peak_db;                 /* in-focus peak, 10*log10f(P+1e-20) */
    float signal_power_db;             /* focus-window mean power, dB */
    int32_t valid;                     /* nRef >= 2 (fft_process.cpp:218-225) */
    int32_t n_ref_windows;             /* reference windows collected */
} sdrg_frame_record;

/* Callback table mirroring the JNI read() callbacks (SDRBridge.kt:141-154,
 * sdr-bridge-java-soapy.cpp:625-693).  Any entry may be NULL.  `stream` is the stream index in the
 * batch.  The order of invocation per frame is soapyCallback's (sdr-bridge-java-soapy.cpp:458-475):
 * fft, detection_flag, mean_snr, mean_snr_sigma, peak_frequency, peak_above_noise_mean, max_bin,
 * best1khz, noise_level; pcm comes from the SSB worker (ssb_processor.cpp:103-113) and is invoked
 * after them, only when the frame produced samples.  spectral_pulse follows noise_level (:477-488, only
 * with SDRG_STAGE_SPECTRAL_PULSE); audio_pulse follows pcm (ssb_processor.cpp:109-113, every frame, only with
 * SDRG_STAGE_AUDIO_PULSE). */
typedef struct sdrg_callbacks {
    void *user;
    void (*fft)(void *user, int32_t stream, const float *power_shifted, int32_t n);        /* ([F)V  */
    void (*detection_flag)(void *user, int32_t stream, int32_t flag);                     /* (I)V   */
    void (*mean_snr)(void *user, int32_t stream, float mean_snr_db);                      /* (F)V   */
    void (*mean_snr_sigma)(void *user, int32_t stream, float mean_snr_sigma);             /* (F)V   */
    void (*peak_frequency)(void *user, int32_t stream, int64_t hz);                       /* (J)V   */
    void (*pcm)(void *user, int32_t stream, const int16_t *pcm, int32_t n);               /* ([S)V  */
    void (*peak_above_noise_mean)(void *user, int32_t stream, float db);                  /* (F)V   */
    void (*max_bin)(void *user, int32_t stream, float snr_db, float snr_sigma);           /* (FF)V  */
    void (*best1khz)(void *user, int32_t stream, float snr_db, float snr_sigma);          /* (FF)V  */
    void (*noise_level)(void *user, int32_t stream, float per_bin_mean);                  /* (F)V   */
    /* (FIJ)V: this frame's best1kHzSnrSigma, SpectralPulseDetector::liveEtat(), llround(estimatedFreqHz()) */
    void (*spectral_pulse)(void *user, int32_t stream, float snr_sigma, int32_t live_etat, int64_t freq_hz);
    /* (FI)V: AudioPulseDetector::lastPulseStrength(), liveEtat() */
    void (*audio_pulse)(void *user, int32_t stream, float strength, int32_t live_etat);
} sdrg_callbacks;

/* Per-kernel device times of the last process call, from hipEvents recorded on the stream each
 * kernel was launched on (only filled while profiling is enabled).  Pipelined, the SSB chain's start marker
 * would sit on the SSB stream, the step's critical path, so a pipelined call carries one only when the call before
 * it was not a profiled SSB call (the first call after a reset of the timing statistics, after profiling was
 * re-enabled, or after an unprofiled call); every other pipelined call's ssb_ms is the interval from the previous
 * call's SSB end marker to its own.  That interval is the SSB chain's own time (its kernels + the launch gaps
 * between them) in SDRG_PIPELINE_INPUTS_READY mode with the host keeping ahead of the GPU.  In SDRG_PIPELINE_ON
 * mode each call's SSB stream first waits for the call's start marker on the main stream, so the interval also
 * holds that wait (the step period rather than the chain), and in any mode it holds the time the host spends
 * blocked between two calls.  The audio pulse detector runs after the chain on a stream of its own. */
typedef struct sdrg_timings {
    float spectrum_ms;   /* unpack + FFT + |X|^2 + fftshift kernel */
    float stats_ms;      /* end of the spectrum -> end of the signal-strength kernel (+ spectral pulse detector when
                            requested), on the statistics' stream; never includes the SSB stream's work */
    float ssb_ms;        /* whole SSB chain (all its kernels; not the audio pulse detector, which runs on a stream
                            of its own after it); pipelined: the SSB stream's time per call, above */
    float total_ms;      /* call start -> end of the main stream's work; joined calls include the SSB stream */
} sdrg_timings;

/* ------------------------------------------------------------------------------------------------
 * Beacon pulse detectors.  One detector per stream, state in HBM, one wavefront per stream per frame:
 *   SpectralPulseDetector  src/dsp/spectral_pulse_detector.h:19-79, .cpp:1-196   (kind SDRG_PULSE_SPECTRAL)
 *     fed one (snrSigma, freqHz) pair per FFT frame (sdr-bridge-java-soapy.cpp:477-479)
 *   AudioPulseDetector     src/ssb/audio_pulse_detector.h:15-104, .cpp:1-256    (kind SDRG_PULSE_AUDIO)
 *     fed each SSB frame's PCM (ssb_processor.cpp:109)
 * Both run the reference's ROI / phase-lock / live-state logic with the same float (and, for the spectral
 * frequency estimate, double) operation order, so outputs are bit-identical to the reference classes.
 * ---------------------------------------------------------------------------------------------- */
enum { SDRG_PULSE_SPECTRAL = 0, SDRG_PULSE_AUDIO = 1 };

/* Union of SpectralPulseDetector::Config (spectral_pulse_detector.h:23-35) and AudioPulseDetector::Config
 * (audio_pulse_detector.h:19-37); sdrg_pulse_config_default() fills the reference defaults of a kind. */
typedef struct sdrg_pulse_config {
    float fs_energy;        /* energy frame rate, Hz (spectral 20, set to fs/N by applyConfig; audio 100) */
    float z_default_s;      /* local-max half-width while unlocked, s (0.666) */
    float t_target_init;    /* initial period, s (1.75) */
    float dt_tol_s;         /* rhythm / lock tolerance, s (0.150) */
    float snr_min;          /* spectral 1.5, audio 1.0 */
    float snr_rhythm;       /* spectral 2.5, audio 1.1 */
    float snr_strong;       /* spectral 4.0, audio 2.0 */
    float dispersion_max;   /* 1.3 */
    int32_t sum_n_max;      /* 7 */
    float live_window_t;    /* live-state look-back in periods (4.0) */
    float live_divisor;     /* 3.0 */
    /* audio front end only */
    float sample_rate;      /* PCM rate the filters are designed for (48000) */
    float f_min, f_max;     /* band-pass edges, Hz (1500, 4000) */
    float smooth_cutoff;    /* energy low-pass, Hz (5) */
    int32_t noise_ref_far;  /* noise reference [i-far, i-near) in energy frames (80, 40) */
    int32_t noise_ref_near;
} sdrg_pulse_config;

/* What the reference getters return after a frame (spectral_pulse_detector.h:41-48,
 * audio_pulse_detector.h:45-49), plus the callback arguments. */
typedef struct sdrg_pulse_output {
    float strength;            /* lastPulseStrength(): snr of the last admitted ROI */
    int32_t live_etat;         /* liveEtat(), 0..5 */
    int32_t level;             /* pulseDetected(): 0 NONE, 1 LOW, 2 MEDIUM, 3 STRONG */
    int32_t locked;            /* isLocked() */
    float period_s;            /* lockedPeriodS() */
    float est_freq_hz;         /* estimatedFreqHz() (spectral; 0 for audio) */
    int64_t est_freq_hz_rounded;  /* std::llround(estimatedFreqHz()), the spectralPulse callback's J */
    float input;               /* spectral: the snrSigma fed this frame (the callback's F); audio: strength */
    int32_t n_energy;          /* energy frames held (diagnostic) */
    int32_t n_rois;            /* ROIs held (diagnostic) */
    int32_t overflow;          /* ROI ring overflows (always 0 within the documented bound; diagnostic) */
} sdrg_pulse_output;

typedef struct sdrg_pulse_bank sdrg_pulse_bank;

/* Reference defaults of a detector kind. */
int32_t sdrg_pulse_config_default(int32_t kind, sdrg_pulse_config *out);
/* n_streams detectors of one kind on HIP device `device` (the reference constructor per stream). */
int32_t sdrg_pulse_bank_create(int32_t kind, const sdrg_pulse_config *cfg, int32_t n_streams, int32_t device,
                               sdrg_pulse_bank **out);
int32_t sdrg_pulse_bank_destroy(sdrg_pulse_bank *bank);
/* SPECTRAL: SpectralPulseDetector::configure (cfg replaced, detector state kept, :6-8).
 * AUDIO: a fresh AudioPulseDetector(cfg) per stream (what SSBProcessor::setPulseConfig does,
 * ssb_processor.cpp:70-95).  Applied in stream order with the process calls. */
int32_t sdrg_pulse_bank_configure(sdrg_pulse_bank *bank, const sdrg_pulse_config *cfg);
int32_t sdrg_pulse_bank_get_config(const sdrg_pulse_bank *bank, sdrg_pulse_config *out);
/* reset() of every detector (spectral_pulse_detector.cpp:179-196, audio_pulse_detector.cpp:242-256). */
int32_t sdrg_pulse_bank_reset(sdrg_pulse_bank *bank);
/* SPECTRAL, one frame per stream, device pointers: stream s reads *(float*)((char*)snr_sigma + s*stride_bytes)
 * and the same for freq_hz (so an sdrg_frame_record array can be passed directly); out: [n_streams]. */
int32_t sdrg_pulse_bank_process_spectral_device(sdrg_pulse_bank *bank, const float *snr_sigma,
                                                const float *freq_hz, int32_t stride_bytes,
                                                sdrg_pulse_output *out);
/* AUDIO, one PCM block per stream, device pointers: stream s has n samples at audio + s*stride samples;
 * sample_format 0 = int16 (process(vector<int16_t>), scaled by 1/32767), 1 = float (process(vector<float>)). */
int32_t sdrg_pulse_bank_process_audio_device(sdrg_pulse_bank *bank, const void *audio, int32_t sample_format,
                                             int32_t n, int32_t stride, sdrg_pulse_output *out);
/* Host-memory variants: copy in, run, copy out, synchronise. */
int32_t sdrg_pulse_bank_process_spectral_host(sdrg_pulse_bank *bank, const float *snr_sigma, const float *freq_hz,
                                              sdrg_pulse_output *out);
int32_t sdrg_pulse_bank_process_audio_host(sdrg_pulse_bank *bank, const void *audio, int32_t sample_format,
                                           int32_t n, sdrg_pulse_output *out);
int32_t sdrg_pulse_bank_synchronize(sdrg_pulse_bank *bank);
/* Run the device-pointer calls on the caller's HIP stream (a hipStream_t; NULL = the bank's own stream). */
int32_t sdrg_pulse_bank_set_stream(sdrg_pulse_bank *bank, void *hip_stream);

/* ------------------------------------------------------------------------------------------------
 * Ingest: exact-N re-chunking of raw device reads (rx_reading_thread, sdr-bridge-java-soapy.cpp:503-575).
 * Reads of any length are appended per stream (accBuffer); every exact samples_per_reading block becomes a
 * frame in a per-stream queue of at most queue_max frames, the oldest dropped when full (RX_QUEUE_MAX = 20,
 * :121, :556-564).  Frames are popped one per stream into a [n_streams][N] batch in the engine format
 * (sdrg_ingest_output_format: the input format, except CS12 which is repacked to CS16).  Host-only.
 * ---------------------------------------------------------------------------------------------- */
typedef struct sdrg_ingest sdrg_ingest;
int32_t sdrg_ingest_create(int32_t n_streams, int32_t samples_per_reading, int32_t in_format, int32_t queue_max,
                           sdrg_ingest **out);
int32_t sdrg_ingest_destroy(sdrg_ingest *ing);
int32_t sdrg_ingest_output_format(const sdrg_ingest *ing);
/* readStream() returned n_samples complex samples in the input format for `stream` */
int32_t sdrg_ingest_push(sdrg_ingest *ing, int32_t stream, const void *raw, int64_t n_samples);
/* queued frames, samples of the partial frame, frames dropped from a full queue so far */
int32_t sdrg_ingest_status(const sdrg_ingest *ing, int32_t stream, int32_t *queued, int32_t *partial_samples,
                           int64_t *dropped_frames);
/* when every stream has a queued frame: pop one per stream into out [n_streams][N] and set *popped = 1;
 * otherwise *popped = 0 and nothing changes */
int32_t sdrg_ingest_pop_batch(sdrg_ingest *ing, void *out, int32_t *popped);
/* one stream's oldest frame (rx_process_thread's pop, :597-603) */
int32_t sdrg_ingest_pop(sdrg_ingest *ing, int32_t stream, void *out, int32_t *popped);
/* setSamplesPerReading: cut at n from now on (queued frames of the old size are discarded) */
int32_t sdrg_ingest_set_samples_per_reading(sdrg_ingest *ing, int32_t n);

/* ------------------------------------------------------------------------------------------------
 * SSBProcessor (src/ssb/ssb_processor.h:24-58, ssb_processor.cpp:26-115): the reference runs the SSB chain on a
 * worker thread fed by soapyCallback through a queue of at most 3 frames that drops its OLDEST frame when full
 * (:51-64); per popped frame, processSSB_opt with the frame's sample rate and the current sound mode, then the
 * PCM callback (only when the frame produced samples), then the audio pulse detector and its callback (:77-115).
 * This object is that worker over a one-stream engine (SSB + audio-pulse stages), so a consumer that falls behind
 * drops the same frames as the reference and the filter state continues over the frames that were processed.
 * Callbacks run on the worker thread.
 * ---------------------------------------------------------------------------------------------- */
typedef struct sdrg_ssb_processor sdrg_ssb_processor;
typedef struct sdrg_ssb_callbacks {
    void *user;
    void (*pcm)(void *user, const int16_t *pcm, int32_t n);                     /* pcmCallback, ([S)V */
    void (*pulse)(void *user, float strength, int32_t live_etat);               /* pulseCallback_, (FI)V */
} sdrg_ssb_callbacks;
/* queue_max: frames held before the oldest is dropped (0 = the reference's 3). */
int32_t sdrg_ssb_processor_create(int32_t device, int32_t queue_max, sdrg_ssb_processor **out);
int32_t sdrg_ssb_processor_destroy(sdrg_ssb_processor *p);   /* stopProcessing + release */
int32_t sdrg_ssb_processor_start(sdrg_ssb_processor *p, const sdrg_ssb_callbacks *cbs);  /* startProcessing */
int32_t sdrg_ssb_processor_stop(sdrg_ssb_processor *p);      /* stopProcessing: the worker finishes its frame */
/* enqueueData: copies the frame (n samples in `format`) with the rate it was read at; ignored when not started. */
int32_t sdrg_ssb_processor_enqueue(sdrg_ssb_processor *p, const void *iq, int32_t format, int32_t n,
                                   int64_t sample_rate);
/* BridgeConfig::getSoundMode() as the worker reads it per frame (:102); default 1. */
int32_t sdrg_ssb_processor_set_sound_mode(sdrg_ssb_processor *p, int32_t mode);
/* setPulseConfig (:70-75): a fresh AudioPulseDetector with cfg before the next frame. */
int32_t sdrg_ssb_processor_set_pulse_config(sdrg_ssb_processor *p, const sdrg_pulse_config *cfg);
float sdrg_ssb_processor_get_ambient_energy(const sdrg_ssb_processor *p);  /* getAmbientEnergy (ssb_processor.h:34) */
float sdrg_ssb_processor_get_current_ratio(const sdrg_ssb_processor *p);   /* getCurrentRatio (:35): always 0 */
/* Wait until the queue is empty and the worker idle (or stopped). */
int32_t sdrg_ssb_processor_drain(sdrg_ssb_processor *p);
/* Frames enqueued, dropped from a full queue, processed; status of the last failed frame (0 if none). */
int32_t sdrg_ssb_processor_counters(const sdrg_ssb_processor *p, int64_t *enqueued, int64_t *dropped,
                                    int64_t *processed, int32_t *last_status);

typedef struct sdrg_engine sdrg_engine;

/* Library identity. */
int32_t sdrg_abi_version(void);
const char *sdrg_last_error(void);      /* thread-local message for the last failing call */

/* Geometry helpers (host-only, no device needed). */
/* Frame size the SSB chain emits for a frame of n samples at sample_rate (0 if none):
 * (n - taps)/decim + 1 with taps = 255 (or n|1 when n < 255), decim = max(1, int(fs/48000.0f))
 * (ssb_demod_opt.cpp:121-143, :273). */
int32_t sdrg_ssb_pcm_len(int32_t n, int64_t sample_rate);

/* The focus window of evaluateSignalStrength (fft_process.cpp:124-140) in the fftshifted spectrum the engine
 * writes: bins [*first_bin, *first_bin + *n_bins) hold offsets -focus_khz .. +focus_khz kHz around the
 * centre.  *n_bins = 0 when the window is empty (focus wider than the band, :218-247).  Host-only; used to
 * gather only the spectrum slice a consumer looks at (sdrg/shard.py gather_focus). */
int32_t sdrg_focus_window(int64_t sample_rate, int32_t n, int32_t focus_khz, int32_t *first_bin, int32_t *n_bins);

/* The SSB filter design the engine uses for a configuration, from the reference's own expressions:
 * rfFilter low-pass (iir2InitLowpass at (float)fs with the sound mode's fc/Q, ssb_demod_opt.cpp:60-73, :262),
 * HP/BP biquads (:148-175, :278-279) and the FIR taps (:121-134).  lpf/hp/bp: {a0, a1, a2, b1, b2};
 * taps must hold 255 floats; *n_taps receives the tap count.  Host-only. */
int32_t sdrg_ssb_design(int32_t samp_count, int64_t sample_rate, int32_t sound_mode, float *lpf, float *hp,
                        float *bp, float *taps, int32_t *n_taps);

/* Page-locked host memory (hipHostMalloc) for sdrg_engine_process_host's buffers: copies to and from it run at
 * the PCIe rate, while pageable buffers go through the runtime's staging.  The memory
 * stays valid until sdrg_host_free; any engine may use it. */
int32_t sdrg_host_alloc(size_t bytes, void **out);
int32_t sdrg_host_free(void *p);

/* Create an engine for n_streams independent receivers on HIP device `device`.
 * Replaces FFTProcessor() + configure() (fft_process.cpp:8-39) and BridgeConfig::initialize
 * (bridge-config.h:17-38) for each stream. */
int32_t sdrg_engine_create(const sdrg_config *cfg, int32_t n_streams, int32_t device, sdrg_engine **out);
int32_t sdrg_engine_destroy(sdrg_engine *eng);

/* JNI applyConfig (sdr-bridge-java-soapy.cpp:1073-1141): BridgeConfig::initialize + FFTProcessor::configure.
 * Per-stream tracking/detection/SSB state is kept, exactly as the reference keeps its members and
 * statics across applyConfig. */
int32_t sdrg_engine_apply_config(sdrg_engine *eng, const sdrg_config *cfg);
/* JNI setFrequency (:878-913): reconfigure + raise isCenterFrequencyChanged for every stream. */
int32_t sdrg_engine_set_frequency(sdrg_engine *eng, int64_t center_frequency);
/* JNI setFrequencyFocusRange (:1025-1040). */
int32_t sdrg_engine_set_frequency_focus_range(sdrg_engine *eng, int32_t khz);
/* JNI setSampleRate (:931-953): BridgeConfig only.  The SSB chain uses the new rate from the next frame (it is
 * handed BridgeConfig's rate per frame, :441-442); the statistics keep the rate of the last configure() point
 * (create / applyConfig / setFrequency / setFrequencyFocusRange), as FFTProcessor::config_ does.  The spectral
 * pulse detector is not reconfigured (only applyConfig does that, :1130-1138). */
int32_t sdrg_engine_set_sample_rate(sdrg_engine *eng, int64_t sample_rate);
/* JNI setSamplesPerReading (:1015-1021): BridgeConfig only; the frame size of the following calls (the reader cuts
 * frames at it, :541-573, and FFTProcessor::process plans whatever length it is handed, fft_process.cpp:42-79). */
int32_t sdrg_engine_set_samples_per_reading(sdrg_engine *eng, int32_t n);
/* JNI setSoundMode (:1066-1071). */
int32_t sdrg_engine_set_sound_mode(sdrg_engine *eng, int32_t mode);
/* processSSB_opt's upperSideband argument (default 1, which is what SSBProcessor always passes,
 * ssb_processor.cpp:103; 0 gives the reference's lower-sideband result, Re - Im of {y, y} = 0). */
int32_t sdrg_engine_set_upper_sideband(sdrg_engine *eng, int32_t upper);
/* BUILD EXTENSION, not a reference interface (BASELINE.json configs[2], "SSB (USB) NCO + FIR-decimate, 127-tap
 * FIR"; the reference chain has neither, ssb_demod_opt.cpp:122).  Off by default, and
 * every reference-parity result above assumes it off.
 *   nco_hz   : != 0 mixes each stream's IQ with a phase-continuous NCO before the chain: sample t of a call
 *              becomes Re((I + jQ) e^{-j 2 pi ph / 2^32}), ph = phase + inc t (mod 2^32), inc =
 *              round(nco_hz / sample_rate * 2^32) mod 2^32; the phasor is hi[ph >> 22] * lo[(ph >> 12) & 1023]
 *              from two 1024-entry tables of e^{-j 2 pi k / 2^10} and e^{-j 2 pi k / 2^20} rounded to float.
 *              The signal at +nco_hz lands at 0 Hz, where removeDC, the low-pass, AGC, FIR and EQ then run
 *              unchanged.  phase starts at 0 and advances by inc * samp_count per call (every stream of the
 *              engine sees the same calls).  0 = no mixer (the reference chain).
 *   fir_taps : decimating FIR length, odd in [3, 255] (Hann-sinc of :121-134 at that length); 0 = 255.
 *              The PCM frame length follows (sdrg_engine_pcm_len).
 * Takes effect at the next call; restarts the NCO phase; filter state is kept. */
int32_t sdrg_engine_set_ssb_variant(sdrg_engine *eng, double nco_hz, int32_t fir_taps);
/* The variant in force: nco_hz, the FIR length the next call uses, the NCO increment and the next call's
 * starting phase (any pointer may be NULL). */
int32_t sdrg_engine_get_ssb_variant(const sdrg_engine *eng, double *nco_hz, int32_t *fir_taps,
                                    uint32_t *nco_increment, uint32_t *nco_phase);
/* Current configuration (BridgeConfig getters, bridge-config.h:41-51). */
int32_t sdrg_engine_get_config(const sdrg_engine *eng, sdrg_config *out);
int32_t sdrg_engine_n_streams(const sdrg_engine *eng);
/* Samples per frame the SSB chain of every stream emits (constant for a configuration). */
int32_t sdrg_engine_pcm_len(const sdrg_engine *eng);

/* The engine's pulse detectors (one SPECTRAL and one AUDIO detector per stream, run by the
 * SDRG_STAGE_SPECTRAL_PULSE / SDRG_STAGE_AUDIO_PULSE stages).  applyConfig sets the spectral detector to
 * the default config with fs_energy = (float)sample_rate / (float)samples_per_reading
 * (sdr-bridge-java-soapy.cpp:1130-1138); create does the same.  set_spectral_pulse_config = configure();
 * set_audio_pulse_config = SSBProcessor::setPulseConfig (fresh detectors at the next frame). */
int32_t sdrg_engine_set_spectral_pulse_config(sdrg_engine *eng, const sdrg_pulse_config *cfg);
int32_t sdrg_engine_set_audio_pulse_config(sdrg_engine *eng, const sdrg_pulse_config *cfg);
/* Device arrays [n_streams] the last process call wrote (valid until the next call; either may be NULL). */
int32_t sdrg_engine_pulse_outputs(const sdrg_engine *eng, const sdrg_pulse_output **spectral,
                                  const sdrg_pulse_output **audio);

/* Reset every stream's cross-frame state (tracking latch, detection ring, SSB filter state, pulse
 * detectors) to the state of a freshly constructed reference process. */
int32_t sdrg_engine_reset_state(sdrg_engine *eng);

/* Process one frame of every stream, all buffers in device memory (HBM).
 *   iq       : [n_streams][samples_per_reading] samples in `format`
 *   spectra  : [n_streams][samples_per_reading] float, fftshifted linear power (fftCallback payload);
 *              may be NULL when STATS is not requested (then an internal buffer is used).  Odd N: element
 *              N-1 of each row is never written, as in the reference's fftshift loop (fft_process.cpp:92-97),
 *              whose member vector keeps its old value there (0 when fresh); a caller buffer should be zeroed
 *              once before its first use, since the statistics may read that bin
 *   records  : [n_streams] sdrg_frame_record (may be NULL if STATS not requested)
 *   pcm      : [n_streams][pcm_len] int16 (may be NULL if SSB not requested)
 *   now_ms   : monotonic clock in ms for the 300 ms frequency-tracking latch
 *              (fft_process.cpp:333-361 uses steady_clock; injected here so results are reproducible)
 * Work is enqueued on the engine's HIP streams and is complete when sdrg_engine_synchronize returns. */
int32_t sdrg_engine_process_device(sdrg_engine *eng, const void *iq, int32_t format, int32_t stages,
                                   float *spectra, sdrg_frame_record *records, int16_t *pcm,
                                   int64_t now_ms);
int32_t sdrg_engine_synchronize(sdrg_engine *eng);
/* evaluateSignalStrength alone (fft_process.cpp:122-379) on caller spectra: [n_streams][samples_per_reading]
 * fftshifted linear power (the FFTProcessor's power_shifted member after process()), records out, each stream's
 * statistics state (tracking latch, detection ring, stale outputs) advanced exactly as by a process() call with
 * STATS.  _device: both buffers in device memory, ordered on the main stream (complete after
 * sdrg_engine_synchronize).  _host: host buffers, synchronous. */
int32_t sdrg_engine_signal_strength_device(sdrg_engine *eng, const float *spectra, sdrg_frame_record *records,
                                           int64_t now_ms);
int32_t sdrg_engine_signal_strength_host(sdrg_engine *eng, const float *spectra, sdrg_frame_record *records,
                                         int64_t now_ms);
/* Enqueue the engine's work on the caller's HIP stream (a hipStream_t; NULL = the engine's own stream): the
 * SSB fork/join happens relative to it, so consumers on that stream (e.g. an RCCL gather of the records)
 * are ordered after each call without a host synchronisation.  Synchronises the previous stream first.
 * The stream must outlive the engine (or be unset with NULL before it is destroyed). */
int32_t sdrg_engine_set_stream(sdrg_engine *eng, void *hip_stream);
/* Pipelining across calls (default SDRG_PIPELINE_OFF).  Pipelined, sdrg_engine_process_device forks the SSB
 * stages at the start of each call and does not join them into the main stream at its end, so a call's SSB
 * pipeline runs beside the next call's spectrum.  The spectrum / statistics / spectral-pulse outputs are
 * ordered on the main stream as usual; the PCM and audio-pulse outputs are complete after
 * sdrg_engine_synchronize (or after the next call's SSB stage starts, which follows them on the SSB stream).
 * process_host always joins.  The input buffer stays in use until the SSB stage has read it: see
 * sdrg_engine_input_released below.
 *   SDRG_PIPELINE_ON: the SSB stage of a call starts after the work enqueued on the main stream before the
 *     call (the caller's producer work on iq), as the spectrum does.
 *   SDRG_PIPELINE_INPUTS_READY: the caller guarantees that iq is complete when the call is made (written by
 *     host-synchronised copies or earlier, already-finished work, e.g. a resident ring of input frames); the
 *     SSB stage then does not wait for the main stream at all, which saves its stream one cross-stream wait
 *     per call.  Work the caller enqueues on the main stream that writes iq is NOT waited for in this mode.
 * SDRG_PIPELINE_STATS_ASYNC may be added (OR) to ON or INPUTS_READY: a call's statistics and spectral pulse detector
 *   run on a stream of their own after the call's spectrum, beside the next call's spectrum, instead of after it
 *   on the main stream.  Every stage of every call still runs, in order per stream; the records and spectral-pulse
 *   outputs are complete after sdrg_engine_synchronize, or on a stream after sdrg_engine_wait_outputs.  The engine
 *   keeps the spectra a call's statistics read intact (a call writing the previous call's spectra buffer waits for
 *   those statistics on the GPU; the host waits for the statistics of the call two before), so a caller rotating
 *   two or more spectra buffers (and records buffers it reads back) overlaps the statistics fully.
 * Any other value returns SDRG_E_INVALID. */
enum { SDRG_PIPELINE_OFF = 0, SDRG_PIPELINE_ON = 1, SDRG_PIPELINE_INPUTS_READY = 2, SDRG_PIPELINE_STATS_ASYNC = 4 };
int32_t sdrg_engine_set_pipelining(sdrg_engine *eng, int32_t mode);
/* Enqueue on `hip_stream` (NULL = the engine's main stream) a wait for every output of the last call: spectra,
 * records and spectral-pulse outputs, PCM and audio-pulse outputs, whichever streams produce them (a consumer of a
 * pipelined call's outputs, e.g. an RCCL gather of the records, then follows them without a host synchronisation). */
int32_t sdrg_engine_wait_outputs(sdrg_engine *eng, void *hip_stream);
/* The INPUT of a call: the kernels read `iq` asynchronously after sdrg_engine_process_device returns -- the
 * spectrum on the main stream and the SSB pipeline on its own stream, which in pipelined mode runs on past the
 * call, beside the next call's spectrum.  The caller must not overwrite or free `iq` until the call has released
 * it.  input_released: *released = 1 once every kernel of the last call that reads its iq has finished (a
 * non-blocking query).  wait_input_released: enqueue on `hip_stream` (NULL = the engine's main stream) a wait for
 * that release, so a refill of the same buffer enqueued there afterwards (e.g. the next frame's host-to-device
 * copy) cannot overtake the readers -- without a host synchronisation and without joining the SSB stream into the
 * next call's spectrum (neither call is needed with a fresh buffer per call). */
int32_t sdrg_engine_input_released(const sdrg_engine *eng, int32_t *released);
int32_t sdrg_engine_wait_input_released(sdrg_engine *eng, void *hip_stream);

/* Same from host memory (PCIe-inclusive): copies iq in, runs, copies outputs back, synchronises,
 * then invokes the registered callbacks per stream in soapyCallback order.  Any output may be NULL. */
int32_t sdrg_engine_process_host(sdrg_engine *eng, const void *iq, int32_t format, int32_t stages,
                                 float *spectra, sdrg_frame_record *records, int16_t *pcm,
                                 int64_t now_ms);
/* Host copies of the last call's pulse outputs ([n_streams] each; either may be NULL); synchronises. */
int32_t sdrg_engine_get_pulse_outputs(sdrg_engine *eng, sdrg_pulse_output *spectral, sdrg_pulse_output *audio);

/* JNI read(): register the callback table (copied). NULL clears it. */
int32_t sdrg_engine_set_callbacks(sdrg_engine *eng, const sdrg_callbacks *cbs);

/* Profiling: when enabled, every process call records hipEvents around each kernel group (a ring of
 * event sets, so back-to-back calls are timed without host synchronisation). */
int32_t sdrg_engine_set_profiling(sdrg_engine *eng, int32_t enabled);
/* Timings of the most recent profiled call (waits for it to finish). */
int32_t sdrg_engine_get_timings(const sdrg_engine *eng, sdrg_timings *out);
/* Mean timings over every profiled call since the last reset (waits for them); *count = calls averaged. */
int32_t sdrg_engine_get_timing_stats(const sdrg_engine *eng, sdrg_timings *mean, int32_t *count);
int32_t sdrg_engine_reset_timing_stats(sdrg_engine *eng);

/* ------------------------------------------------------------------------------------------------
 * Multi-GPU: one process per GPU (rank), each with its own engine for its block of streams (rank r owns the
 * global streams [r*B, (r+1)*B): frames and per-stream state are independent, so nothing else is exchanged), and
 * the per-frame results gathered to a root rank with RCCL (ncclGather over xGMI).  The reference is one receiver
 * in one process; what is gathered is what its soapyCallback hands to Kotlin per frame
 * (sdr-bridge-java-soapy.cpp:456-466: the fftCallback spectrum, the getters' values with the peak) and the SSB
 * worker's PCM (ssb_processor.cpp:103-108).  RCCL is loaded at run time (librccl.so.1) by the first call below;
 * without it they return SDRG_E_UNSUPPORTED and nothing else is affected.
 * ---------------------------------------------------------------------------------------------- */
#define SDRG_DIST_ID_BYTES 128
typedef struct sdrg_dist sdrg_dist;
/* ncclGetUniqueId, on one rank: the caller hands these bytes to every rank (a file, a socket, MPI, ...). */
int32_t sdrg_dist_unique_id(void *id, int32_t bytes);
/* ncclCommInitRank on `device` (collective: every rank of the job calls it with the same id). */
int32_t sdrg_dist_create(const void *id, int32_t world_size, int32_t rank, int32_t device, sdrg_dist **out);
int32_t sdrg_dist_destroy(sdrg_dist *d);
/* Rank, world size, the RCCL version in use and whether the gathers move their bytes through RCCL (1) or, for a
 * one-rank communicator, as hipMemcpyAsync device copies (0).  Any pointer may be NULL. */
int32_t sdrg_dist_info(const sdrg_dist *d, int32_t *rank, int32_t *world_size, int32_t *rccl_version,
                       int32_t *rccl_data);
/* A one-rank communicator's gathers are device copies by default (RCCL's one-rank gather kernel runs beside the SSB
 * pipeline and slows the step: DESIGN.md §7); on = 1 routes them through ncclGather as at world size > 1. */
int32_t sdrg_dist_set_one_rank_rccl(sdrg_dist *d, int32_t on);

/* What one gather moves.  Each selected pair gathers this rank's n_streams rows to the root's output, which
 * holds world_size x n_streams rows in rank order (= global stream order); the *_out pointers are read on the
 * root only (NULL elsewhere).  A NULL source skips the pair; every rank selects the same pairs.  All device memory
 * of the engine's device.
 *   records       [n_streams] sdrg_frame_record  -> records_out [world][n_streams]
 *   focus_spectra [n_streams][N] (a call's spectra) -> focus_out [world][n_streams][n_bins]: each frame's focus
 *                 window (sdrg_focus_window of the statistics' configuration), packed on the device first
 *   spectra       [n_streams][N]                 -> spectra_out [world][n_streams][N]: the whole fftshifted spectra
 *                 (268 MB per rank at 4096 x 16384)
 *   pcm           [n_streams][pcm_len] int16     -> pcm_out [world][n_streams][pcm_len] */
typedef struct sdrg_gather_buffers {
    const sdrg_frame_record *records;
    sdrg_frame_record *records_out;
    const float *focus_spectra;  /* the focus-window slices of these spectra */
    float *focus_out;
    const float *spectra;        /* the whole spectra */
    float *spectra_out;
    const int16_t *pcm;
    int16_t *pcm_out;
} sdrg_gather_buffers;
/* Enqueue the gathers (one RCCL group) behind the last process call's outputs they read, on the engine stream that
 * produced them: the statistics stream when that call ran its statistics asynchronously (its records, and the spectra
 * those statistics waited for), else the main stream; with PCM, the audio detector's stream (after the SSB stage).
 * No host synchronisation; a later call that writes any byte a gather reads (byte ranges overlap: the same buffer, a
 * slice of it, or an offset into it) waits for that gather on the GPU first, and nothing else waits, so a caller
 * rotating its output buffers overlaps the gathers with its next calls.  Every rank calls it with the same selection
 * (the stream choice above depends on it, and RCCL matches the ranks' gathers in issue order).  At world_size > 1 the
 * path is compiled and checked only on one-rank communicators and on the world-2 CPU rehearsal: no two-GPU run has
 * executed it.  Complete after sdrg_engine_synchronize (or on a stream after
 * sdrg_engine_wait_outputs).  Replaces nothing in the reference (one receiver per process): BASELINE configs[3]. */
int32_t sdrg_engine_gather(sdrg_engine *eng, sdrg_dist *d, int32_t root, const sdrg_gather_buffers *bufs);
/* Single-pair forms of sdrg_engine_gather. */
int32_t sdrg_engine_gather_records(sdrg_engine *eng, sdrg_dist *d, int32_t root, const sdrg_frame_record *records,
                                   sdrg_frame_record *records_out);
int32_t sdrg_engine_gather_focus(sdrg_engine *eng, sdrg_dist *d, int32_t root, const float *spectra, float *focus_out);
int32_t sdrg_engine_gather_spectra(sdrg_engine *eng, sdrg_dist *d, int32_t root, const float *spectra,
                                   float *spectra_out);
int32_t sdrg_engine_gather_pcm(sdrg_engine *eng, sdrg_dist *d, int32_t root, const int16_t *pcm, int16_t *pcm_out);

/* Device memory for a host that has no other GPU allocator (the C/C++ side of the JNI boundary): hipMalloc /
 * hipFree on `device`, and a synchronous copy in any direction (hipMemcpyDefault; it is not ordered with the
 * engine's streams -- call sdrg_engine_synchronize before reading an engine output back). */
int32_t sdrg_device_alloc(int32_t device, size_t bytes, void **out);
int32_t sdrg_device_free(int32_t device, void *p);
int32_t sdrg_memcpy(int32_t device, void *dst, const void *src, size_t bytes);
/* Measurement (bench.py's roofline basis, not part of the reference's surface): the read + write GB/s of a float4
 * streaming copy of `bytes` on `device` (nontemporal loads and stores, 16 workgroups per CU, `reps` timed launches
 * after one untimed), the achievable HBM rate a memory-bound kernel is priced against beside the 8 TB/s spec. */
int32_t sdrg_measure_hbm_copy(int32_t device, size_t bytes, int32_t reps, double *gbs);

#ifdef __cplusplus
}
#endif

#endif /* SDRG_H */
