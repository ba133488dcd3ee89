// fftany.h — host side of the any-N spectrum kernels (fftany.hip): the per-N plan, its table layout and
// launcher.  Power-of-two N in [64, 65536] use spectrum.hip's kernels instead (spectrum_supported_pow2).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace sdrg {

// Stockham passes of one sequence length L (radix per pass, product of the earlier radices)
struct FftPassPlan {
    int32_t L;
    int32_t n_pass;
    int32_t radix[16];
    int32_t ns[16];
};

struct AnyPlan {
    enum Mode { ONE = 0, FOUR = 1, BLUE_ONE = 2, BLUE_FOUR = 3 };
    int32_t mode = ONE;
    int32_t n = 0;          // frame size N
    int32_t m = 0;          // transform size (N, or Bluestein's power of two M >= 2N - 1)
    int32_t n1 = 0, n2 = 0; // four-step factors of m
};

AnyPlan any_plan(int n);
size_t any_table_floats(const AnyPlan &p);
void any_fill_tables(const AnyPlan &p, float *out);
size_t any_scratch_floats(const AnyPlan &p, int n_frames);
int any_wave_frames(const AnyPlan &p, int n_frames);
hipError_t launch_spectrum_any(const AnyPlan &p, const void *iq, int fmt, int n_frames, const float *tables,
                               float *spectra, float *scratch, hipStream_t s);

}  // namespace sdrg
