// Host build of the synthetic grid renderer (mantis_amd/csrc/synth.h) for CPU
// tests; the product library carries the HIP kernel build of the same header.
#include <cstdint>

#include "../mantis_amd/csrc/synth.h"

extern "C" void mantis_synth_render_host(const mantis_synth::Cam* cam, uint64_t seed, uint8_t* out) {
  for (int y = 0; y < cam->h; y++)
    for (int x = 0; x < cam->w; x++) mantis_synth::render_pixel(*cam, x, y, seed, out + ((size_t)y * cam->w + x) * 3);
}
