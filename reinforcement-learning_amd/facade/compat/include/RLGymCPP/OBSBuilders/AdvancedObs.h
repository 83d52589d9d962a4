// compat <RLGymCPP/OBSBuilders/AdvancedObs.h>: the declarations restated in facade/RLGC.hpp (device registry classes and builders)
#pragma once
#include "RLGC.hpp"
