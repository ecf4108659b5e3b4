// dcte_emu.cpp -- host emulation of the gfx950 kernel's fp32 arithmetic.
//
// TEST INFRASTRUCTURE.  Runs dcte_passes.h / dcte_math.h (the kernel's own
// code, through dcte_pixel.h) on the CPU, pixel by pixel, so CPU-only tests can measure the fp32
// path's error against the oracle on large and adversarial inputs, and GPU
// tests can demand bit-equality between device and emulation.
#include <math.h>
#include <stddef.h>
#include <stdint.h>

#include "dcte_pixel.h"

using namespace dcte;


extern "C" {

// Per-pixel emulation over rows [y0, y1).  we / wt are the kernel's scaled
// weights; outputs E (the kernel's fast-path value), and the raw m_e / m_t.
int emu_energy_map(const uint8_t* px, int w, int h, int bpp, size_t rowstride, int n,
                   float we, float wt, int sem, int y0, int y1, float* E, float* me_out,
                   float* mt_out)
{
    for (int y = y0; y < y1; y++)
        for (int x = 0; x < w; x++) {
            float mt, me;
            const long long rs = (long long)rowstride;
            switch (n) {
            case 2: pixel_maxima<2>(px, rs, 0, w, h, bpp, sem, x, y, mt, me); break;
            case 4: pixel_maxima<4>(px, rs, 0, w, h, bpp, sem, x, y, mt, me); break;
            case 8: pixel_maxima<8>(px, rs, 0, w, h, bpp, sem, x, y, mt, me); break;
            case 16: pixel_maxima<16>(px, rs, 0, w, h, bpp, sem, x, y, mt, me); break;
            default: return -1;
            }
            size_t k = (size_t)(y - y0) * w + x;
            E[k] = me > mt ? me * we : mt * wt;
            if (me_out) me_out[k] = me;
            if (mt_out) mt_out[k] = mt;
        }
    return 0;
}

// The second (column) pass alone on a ring of row-transform outputs, oldest
// row first: ring[j * CH + k] for N = 2, 4, 8 (CH = N); N = 16 takes the four
// channels of wave q (ring[j * 4 + c], channel c = k1 4c + {0,2,1,3}[q]).
// Returns the pass's (m_t, m_e) in hat units.
int emu_cols(int n, const float* ring, int q, float* mt, float* me)
{
    switch (n) {
    case 2: { float r[2][2]; for (int i = 0; i < 4; i++) r[i / 2][i % 2] = ring[i];
              Cols<2>::run<0>(r, 0, *mt, *me); return 0; }
    case 4: { float r[4][4]; for (int i = 0; i < 16; i++) r[i / 4][i % 4] = ring[i];
              Cols<4>::run<0>(r, 0, *mt, *me); return 0; }
    case 8: { float r[8][8]; for (int i = 0; i < 64; i++) r[i / 8][i % 8] = ring[i];
              Cols<8>::run<0>(r, 0, *mt, *me); return 0; }
    case 16: { float r[16][4]; for (int i = 0; i < 64; i++) r[i / 4][i % 4] = ring[i];
               Cols<16>::run<0>(r, q, *mt, *me); return 0; }
    default: return -1;
    }
}
}
