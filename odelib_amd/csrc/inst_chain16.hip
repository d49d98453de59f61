// instantiation unit: Chain<16>
#include "../../include/odelib_amd.h"
#include "dispatch.h"
OE_DECLARE_ENTRY(chain16) { return oe::make_entry<oe::Chain<16>>(OE_MODEL_CHAIN); }
