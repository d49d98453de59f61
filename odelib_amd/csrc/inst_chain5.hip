// instantiation unit: Chain<5>
#include "../../include/odelib_amd.h"
#include "dispatch.h"
OE_DECLARE_ENTRY(chain5) { return oe::make_entry<oe::Chain<5>>(OE_MODEL_CHAIN); }
