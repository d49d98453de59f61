// instantiation unit: ZeroI
#include "../../include/odelib_amd.h"
#include "dispatch.h"
OE_DECLARE_ENTRY(zero_i) { return oe::make_entry<oe::ZeroI>(OE_MODEL_ZERO_I); }
