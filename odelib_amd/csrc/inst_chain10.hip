// instantiation unit: Chain<10>
#include "../../include/odelib_amd.h"
#include "dispatch.h"
OE_DECLARE_ENTRY(chain10) { return oe::make_entry<oe::Chain<10>>(OE_MODEL_CHAIN); }
