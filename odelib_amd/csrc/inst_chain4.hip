// instantiation unit: Chain<4>
#include "../../include/odelib_amd.h"
#include "dispatch.h"
OE_DECLARE_ENTRY(chain4) { return oe::make_entry<oe::Chain<4>>(OE_MODEL_CHAIN); }
