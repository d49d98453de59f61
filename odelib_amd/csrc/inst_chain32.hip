// instantiation unit: Chain<32>
#include "../../include/odelib_amd.h"
#include "dispatch.h"
OE_DECLARE_ENTRY(chain32) { return oe::make_entry<oe::Chain<32>>(OE_MODEL_CHAIN); }
