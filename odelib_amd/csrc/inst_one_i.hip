// instantiation unit: OneI
#include "../../include/odelib_amd.h"
#include "dispatch.h"
OE_DECLARE_ENTRY(one_i) { return oe::make_entry<oe::OneI>(OE_MODEL_ONE_I); }
