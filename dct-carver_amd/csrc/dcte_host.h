// dcte_host.h -- host helpers shared by dcte_capi.cpp and dcte_host.cpp.
#pragma once

namespace dcte {

// the reference's makect twiddles for ddct2d, n = 2, 4 (else zeros)
void small_twiddles(int n, double ct[4]);

}  // namespace dcte
