// compat <GigaLearnCPP/Learner.h>: GGL::Learner / LearnerConfig / Report of the MI355X trainer facade
#pragma once
#include "GigaLearn.hpp"
