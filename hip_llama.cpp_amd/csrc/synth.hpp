// synth.hpp — product-side include of the shared generator (include/thallama_synth.h).
#pragma once
#include "../../include/thallama_synth.h"
