// compat <RLGymCPP/Rewards/KickoffProximityReward2v2Enhanced.h>: the declarations restated in facade/RLGC.hpp (device registry classes and builders)
#pragma once
#include "RLGC.hpp"
