// instantiation unit: Chain<24>
#include "../../include/odelib_amd.h"
#include "dispatch.h"
OE_DECLARE_ENTRY(chain24) { return oe::make_entry<oe::Chain<24>>(OE_MODEL_CHAIN); }
