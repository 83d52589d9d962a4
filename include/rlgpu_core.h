/*
 * rlgpu_core.h -- error convention and version of the rlgpu C ABI.
 *
 * The reference reports errors by logging and throwing std::runtime_error
 * (RG_ERR_CLOSE, GigaLearnCPP/RLGymCPP/src/RLGymCPP/Framework.h:16-21;
 * RS_ERR_CLOSE, GigaLearnCPP/RLGymCPP/RocketSim/src/Framework.h:67-72).
 * Across this C boundary every entry point instead returns an int status and
 * keeps a thread-local message; the C++ facade (rlgpu.hpp) turns a non-zero
 * status back into std::runtime_error so the Learner's try/catch behaves the
 * same (GigaLearnCPP/src/public/GigaLearnCPP/Learner.cpp:466-474,
 * PPO/PPOLearner.cpp:504-518,571-580).
 */
#ifndef RLGPU_CORE_H
#define RLGPU_CORE_H

#ifdef __cplusplus
extern "C" {
#endif

enum rlgpu_status {
    RLGPU_OK = 0,
    RLGPU_ERR_INVALID_ARG = -1,   /* bad size / null pointer / out-of-range config */
    RLGPU_ERR_HIP = -2,           /* a HIP runtime call failed */
    RLGPU_ERR_OOM = -3,           /* device allocation failed */
    RLGPU_ERR_STATE = -4,         /* call not valid in the handle's current state */
    RLGPU_ERR_UNSUPPORTED = -5    /* plugin / reward / condition type not built */
};

/* Message of the last failing call on this thread ("" if none). */
const char* rlgpu_last_error(void);

/* ABI version: major*10000 + minor*100 + patch. */
int rlgpu_abi_version(void);

/* Number of visible HIP devices (0 if no GPU); never fails. */
int rlgpu_device_count(void);

#ifdef __cplusplus
}
#endif
#endif
