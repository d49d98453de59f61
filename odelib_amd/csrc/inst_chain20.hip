// instantiation unit: Chain<20>
#include "../../include/odelib_amd.h"
#include "dispatch.h"
OE_DECLARE_ENTRY(chain20) { return oe::make_entry<oe::Chain<20>>(OE_MODEL_CHAIN); }
