// instantiation unit: TwoI
#include "../../include/odelib_amd.h"
#include "dispatch.h"
OE_DECLARE_ENTRY(two_i) { return oe::make_entry<oe::TwoI>(OE_MODEL_TWO_I); }
