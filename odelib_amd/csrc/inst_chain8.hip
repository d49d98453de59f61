// instantiation unit: Chain<8>
#include "../../include/odelib_amd.h"
#include "dispatch.h"
OE_DECLARE_ENTRY(chain8) { return oe::make_entry<oe::Chain<8>>(OE_MODEL_CHAIN); }
