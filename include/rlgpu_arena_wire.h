/*
 * rlgpu_arena_wire.h -- RocketSim's arena byte stream for the arena records of rlgpu_env.h.
 * Host code: no GPU work except the envset get / set of the two envset entry points.
 *
 * Replaces (RS/ = GigaLearnCPP/RLGymCPP/RocketSim/src/):
 *   Arena::Serialize(DataStreamOut&)        RS/Sim/Arena/Arena.cpp:572-599  -> rlgpu_arena_serialize
 *   Arena::DeserializeNew(DataStreamIn&)    RS/Sim/Arena/Arena.cpp:601-671  -> rlgpu_arena_deserialize
 *   DataStreamOut::WriteToFile(path, true)  RS/DataStream/DataStreamOut.h:46-59: the file is
 *       u32 RLGPU_RS_VERSION_ID followed by the stream (rlgpu/arena_wire.py to_file / from_file)
 *
 * The stream is the reference's byte for byte: little-endian, WriteMultiple = u32 field count then
 * each field's sizeof(T) bytes (DataStreamOut.h:35-44), with the field lists of Arena, ArenaConfig,
 * Car (controls, config, BallHitInfo, CarState), BoostPadState, BallState and MutatorConfig.
 * Units as Car/Ball::GetState (pos, vel in uu; Car.cpp:10-19, Ball.cpp:27-33); reading applies
 * SetState's * UU_TO_BT (Car.cpp:23-36, Ball.cpp:35-49).
 *
 * The engine simulates SOCCAR 2v2 Octanes at 120 Hz with the default ArenaConfig / MutatorConfig:
 * the writer emits those sections as the reference writes its defaults, and the reader returns
 * RLGPU_ERR_UNSUPPORTED for a stream that asks for anything else (another mode or tick rate, car
 * body, mutator value, custom pads) instead of simulating it with other constants.  Cars are
 * written in id order 1..4 (team = (id - 1) & 1, the order ExampleMain's EnvSet adds them).  A
 * malformed stream (truncated, wrong field count) is RLGPU_ERR_INVALID_ARG, as
 * DataStreamIn::ReadMultipleFromList fails on a count mismatch (DataStreamIn.h:73-80).
 *
 * Reading into a record: every serialized field is written; RocketSim state the stream does not
 * carry is reset as DeserializeNew's new arena has it (is_supersonic, air_time, wheel contacts
 * and wheel values, velocity-impulse caches, ball_sleeping, an invalid BallHitInfo's fields); the
 * RLGym bookkeeping in st->env other than tick_count is left as the caller set it.
 */
#ifndef RLGPU_ARENA_WIRE_H
#define RLGPU_ARENA_WIRE_H

#include <stdint.h>
#include "rlgpu_env.h"

#ifdef __cplusplus
extern "C" {
#endif

/* RS_VERSION_ID of RocketSim "2.1.1" (RS/Framework.h:3,100-106): the u32 WriteToFile prepends. */
#define RLGPU_RS_VERSION_ID 302020u

/* Bytes rlgpu_arena_serialize writes for *st: 2,076 + 68 per car with a valid BallHitInfo. */
int rlgpu_arena_serialized_size(const rlgpu_arena_state* st, uint64_t* out_bytes);

/* Arena::Serialize of one arena record into out[0, cap); *written = bytes written. */
int rlgpu_arena_serialize(const rlgpu_arena_state* st, uint8_t* out, uint64_t cap, uint64_t* written);

/* Arena::DeserializeNew: one arena from in[0, n) into *st; *consumed = bytes read (may be NULL). */
int rlgpu_arena_deserialize(const uint8_t* in, uint64_t n, rlgpu_arena_state* st, uint64_t* consumed);

/* The same on arena `index` of an env set (device record; synchronous).  After a deserialize,
 * rlgpu_envset_build_obs refreshes the arena's obs / mask rows. */
int rlgpu_envset_serialize_arena(rlgpu_envset* env, int32_t index, uint8_t* out, uint64_t cap, uint64_t* written);
int rlgpu_envset_deserialize_arena(rlgpu_envset* env, int32_t index, const uint8_t* in, uint64_t n,
                                   uint64_t* consumed);

#ifdef __cplusplus
}
#endif
#endif
