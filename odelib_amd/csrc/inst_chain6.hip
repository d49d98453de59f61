// instantiation unit: Chain<6>
#include "../../include/odelib_amd.h"
#include "dispatch.h"
OE_DECLARE_ENTRY(chain6) { return oe::make_entry<oe::Chain<6>>(OE_MODEL_CHAIN); }
