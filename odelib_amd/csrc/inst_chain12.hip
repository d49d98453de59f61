// instantiation unit: Chain<12>
#include "../../include/odelib_amd.h"
#include "dispatch.h"
OE_DECLARE_ENTRY(chain12) { return oe::make_entry<oe::Chain<12>>(OE_MODEL_CHAIN); }
