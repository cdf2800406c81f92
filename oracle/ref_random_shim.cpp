// TEST INFRASTRUCTURE ONLY: C entry points into the reference's own
// misc/Random.cpp (compiled unmodified from /root/reference by
// oracle/Makefile), to pin the oracle's scene random numbers
// (rt_oracle.c orc_get_float) against the reference's Random::getFloat /
// Random::init (RayTrace/misc/Random.cpp).
//
// Random.cpp references Log::logW (misc/Log.cpp, which needs SDL and is not
// built here); that call is only reached when Random::init was never called,
// so the library leaves the symbol unresolved and every caller below calls
// ref_random_init first.  No stand-in is provided for it.
#include "misc/Random.h"

extern "C" {
void ref_random_init(unsigned seed) { Random::init(seed); }
float ref_random_get_float(float min, float max) { return Random::getFloat(min, max); }
int ref_random_get_int(int min, int max) { return Random::getInt(min, max); }
}
