// ingest.cpp — exact-N re-chunking of raw device reads into engine frames (host runtime, sdrg_ingest_* C ABI).
//
// The reference's rx_reading_thread (src/sdr-bridge-java-soapy.cpp:503-575) appends every readStream() result
// (any length up to the stream MTU) to accBuffer, cuts it into blocks of exactly samplesPerReading samples,
// and queues each block for rx_process_thread, dropping the OLDEST queued block when RX_QUEUE_MAX = 20 are
// waiting (:121, :556-564).  This does the same per stream for n_streams receivers, and pops one frame of
// every stream at once into a [n_streams][N] batch — the layout sdrg_engine_process_host/_device take.
//
// Formats: the reference's stream is CF32 (:263) and the Soapy drivers convert native samples; the engine
// unpacks CS8 / CU8 / CS16 / CF32 itself, so those pass through as raw bytes.  Packed 12-bit CS12
// (getBytesPerSample: 3 bytes per complex sample, :161-163) is repacked to CS16 with SoapySDR's published
// CS12 -> CS16 layout (I = byte0 | (byte1 & 0x0f) << 8, Q = byte1 >> 4 | byte2 << 4, each placed in the top
// 12 bits of an int16), so the engine's CS16 scale 1/32768 gives the 12-bit value / 2048.  SoapySDR is not
// part of the reference tree, so that convention is unpinned by a reference fixture.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "pulse_bank.h"  // sdrg::fail

using namespace sdrg;

struct sdrg_ingest {
    int n_streams = 0;
    int n = 0;            // samplesPerReading
    int in_fmt = 0;       // format pushed
    int out_fmt = 0;      // format popped (CS12 -> CS16)
    int in_bps = 0, out_bps = 0;
    int queue_max = 20;   // RX_QUEUE_MAX
    struct Stream {
        std::vector<uint8_t> acc;          // accBuffer: partial frame, already in out_fmt (< n samples)
        std::vector<uint8_t> ring;         // queue_max frame slots of n * out_bps bytes
        int head = 0, count = 0;           // queued frames
        int64_t dropped = 0, pushed = 0;   // frames dropped from a full queue / samples pushed
    };
    std::vector<Stream> st;
};

namespace {

int in_bytes_per_sample(int fmt) {
    switch (fmt) {
    case SDRG_IQ_CF32: return 8;
    case SDRG_IQ_CS16: return 4;
    case SDRG_IQ_CS8:
    case SDRG_IQ_CU8: return 2;
    case SDRG_IQ_CS12: return 3;
    default: return 0;
    }
}

// SoapySDR's CS12 -> CS16 (ConverterPrimitives), one complex sample
inline void cs12_to_cs16(const uint8_t *in, int16_t *out) {
    const uint16_t b0 = in[0], b1 = in[1], b2 = in[2];
    out[0] = (int16_t)(uint16_t)((b1 << 12) | (b0 << 4));
    out[1] = (int16_t)(uint16_t)((b2 << 8) | (b1 & 0xf0));
}

void convert(const sdrg_ingest *g, const uint8_t *src, int64_t n, uint8_t *dst) {
    if (g->in_fmt == SDRG_IQ_CS12) {
        int16_t *o = reinterpret_cast<int16_t *>(dst);
        for (int64_t k = 0; k < n; k++) cs12_to_cs16(src + 3 * k, o + 2 * k);
    } else {
        memcpy(dst, src, (size_t)n * (size_t)g->in_bps);
    }
}

// queue one complete frame (rx_queue.push_back, dropping the front when full)
uint8_t *queue_slot(sdrg_ingest *g, sdrg_ingest::Stream &s) {
    const size_t fb = (size_t)g->n * g->out_bps;
    if (s.ring.empty()) s.ring.resize(fb * (size_t)g->queue_max);
    if (s.count == g->queue_max) {
        s.head = (s.head + 1) % g->queue_max;
        s.count--;
        s.dropped++;
    }
    const int slot = (s.head + s.count) % g->queue_max;
    s.count++;
    return s.ring.data() + fb * (size_t)slot;
}

}  // namespace

extern "C" {

int32_t sdrg_ingest_create(int32_t n_streams, int32_t samples_per_reading, int32_t in_format, int32_t queue_max,
                           sdrg_ingest **out) {
    if (!out) return fail(SDRG_E_INVALID, "null out");
    *out = nullptr;
    if (n_streams <= 0 || samples_per_reading <= 0 || samples_per_reading > (1 << 20))
        return fail(SDRG_E_INVALID, "bad n_streams / samples_per_reading");
    if (!in_bytes_per_sample(in_format)) return fail(SDRG_E_INVALID, "unknown input format %d", in_format);
    if (queue_max <= 0) return fail(SDRG_E_INVALID, "queue_max must be > 0");
    sdrg_ingest *g = new sdrg_ingest();
    g->n_streams = n_streams;
    g->n = samples_per_reading;
    g->in_fmt = in_format;
    g->out_fmt = in_format == SDRG_IQ_CS12 ? SDRG_IQ_CS16 : in_format;
    g->in_bps = in_bytes_per_sample(in_format);
    g->out_bps = in_bytes_per_sample(g->out_fmt);
    g->queue_max = queue_max;
    g->st.resize(n_streams);
    *out = g;
    return SDRG_OK;
}

int32_t sdrg_ingest_destroy(sdrg_ingest *g) {
    delete g;
    return SDRG_OK;
}

int32_t sdrg_ingest_output_format(const sdrg_ingest *g) { return g ? g->out_fmt : -1; }

int32_t sdrg_ingest_push(sdrg_ingest *g, int32_t stream, const void *raw, int64_t n_samples) {
    if (!g) return fail(SDRG_E_INVALID, "null ingest");
    if (stream < 0 || stream >= g->n_streams) return fail(SDRG_E_INVALID, "stream %d out of range", stream);
    if (n_samples < 0 || (n_samples > 0 && !raw)) return fail(SDRG_E_INVALID, "bad read");
    sdrg_ingest::Stream &s = g->st[stream];
    const uint8_t *src = static_cast<const uint8_t *>(raw);
    const size_t fb = (size_t)g->n * g->out_bps;
    s.pushed += n_samples;
    int64_t left = n_samples;
    while (left > 0) {
        const int64_t have = (int64_t)(s.acc.size() / g->out_bps);
        const int64_t take = std::min<int64_t>(left, g->n - have);
        if (have == 0 && take == g->n) {  // a whole frame straight from the read
            convert(g, src, take, queue_slot(g, s));
        } else {
            s.acc.resize((size_t)(have + take) * g->out_bps);
            convert(g, src, take, s.acc.data() + (size_t)have * g->out_bps);
            if (have + take == g->n) {
                memcpy(queue_slot(g, s), s.acc.data(), fb);
                s.acc.clear();
            }
        }
        src += (size_t)take * g->in_bps;
        left -= take;
    }
    return SDRG_OK;
}

int32_t sdrg_ingest_status(const sdrg_ingest *g, int32_t stream, int32_t *queued, int32_t *partial_samples,
                           int64_t *dropped_frames) {
    if (!g) return fail(SDRG_E_INVALID, "null ingest");
    if (stream < 0 || stream >= g->n_streams) return fail(SDRG_E_INVALID, "stream %d out of range", stream);
    const sdrg_ingest::Stream &s = g->st[stream];
    if (queued) *queued = s.count;
    if (partial_samples) *partial_samples = (int32_t)(s.acc.size() / g->out_bps);
    if (dropped_frames) *dropped_frames = s.dropped;
    return SDRG_OK;
}

int32_t sdrg_ingest_pop_batch(sdrg_ingest *g, void *out, int32_t *popped) {
    if (!g || !out || !popped) return fail(SDRG_E_INVALID, "null argument");
    *popped = 0;
    for (const auto &s : g->st)
        if (s.count == 0) return SDRG_OK;  // not every stream has a frame yet
    const size_t fb = (size_t)g->n * g->out_bps;
    uint8_t *dst = static_cast<uint8_t *>(out);
    for (int k = 0; k < g->n_streams; k++) {
        sdrg_ingest::Stream &s = g->st[k];
        memcpy(dst + fb * (size_t)k, s.ring.data() + fb * (size_t)s.head, fb);
        s.head = (s.head + 1) % g->queue_max;
        s.count--;
    }
    *popped = 1;
    return SDRG_OK;
}

int32_t sdrg_ingest_pop(sdrg_ingest *g, int32_t stream, void *out, int32_t *popped) {
    if (!g || !out || !popped) return fail(SDRG_E_INVALID, "null argument");
    if (stream < 0 || stream >= g->n_streams) return fail(SDRG_E_INVALID, "stream %d out of range", stream);
    *popped = 0;
    sdrg_ingest::Stream &s = g->st[stream];
    if (s.count == 0) return SDRG_OK;
    const size_t fb = (size_t)g->n * g->out_bps;
    memcpy(out, s.ring.data() + fb * (size_t)s.head, fb);
    s.head = (s.head + 1) % g->queue_max;
    s.count--;
    *popped = 1;
    return SDRG_OK;
}

// setSamplesPerReading: the reader cuts at the new size from its next iteration (:512-514, :550); frames
// already queued at the old size cannot form an N-sample batch and are discarded; the partial accumulation
// is kept (truncated into whole new frames as the reference's while-loop would cut it).
int32_t sdrg_ingest_set_samples_per_reading(sdrg_ingest *g, int32_t n) {
    if (!g) return fail(SDRG_E_INVALID, "null ingest");
    if (n <= 0 || n > (1 << 20)) return fail(SDRG_E_INVALID, "bad samples_per_reading %d", n);
    if (n == g->n) return SDRG_OK;
    const int old_bps = g->out_bps;
    for (auto &s : g->st) {
        std::vector<uint8_t> acc;
        acc.swap(s.acc);
        s.ring.clear();
        s.head = s.count = 0;
        const int64_t have = (int64_t)(acc.size() / old_bps);
        g->n = n;
        // re-push the kept samples through the cutter (already converted: copy as out_fmt bytes)
        const size_t fb = (size_t)n * g->out_bps;
        int64_t off = 0;
        while (have - off >= n) {
            memcpy(queue_slot(g, s), acc.data() + (size_t)off * g->out_bps, fb);
            off += n;
        }
        s.acc.assign(acc.begin() + (size_t)off * g->out_bps, acc.end());
    }
    g->n = n;
    return SDRG_OK;
}

}  // extern "C"
