/*
 * othello_mi355x.h -- C ABI of the MI355X-native vectorised Othello rules engine.
 *
 * Drop-in boundary for the reference's hot path: the
 * in-process Gym-style API of OthelloBaseEnv / SimpleOthelloEnv / OthelloEnv
 * (othello.py:21-501), batched over E boards that live in HBM.  The reference
 * is pure Python and has no FFI of its own, so these entry points are what a
 * ctypes binding of it would call (INTEGRATION.md shows that binding).
 *
 * Each entry point below names the reference function it replaces.
 *
 * Conventions
 *   - All array arguments are DEVICE pointers (hipMalloc / torch.cuda tensors)
 *     unless stated; `stream` is a hipStream_t (NULL = the null stream).  Calls
 *     only enqueue work: nothing synchronises the host.
 *   - Square a = row * N + col (othello.py:392-393); action a in [0, N*N).
 *   - W = ceil(N*N / 64) 64-bit words per colour (1 for N <= 8, up to 4 for N = 16).
 *   - State exchange format (also used by the test oracle):
 *       boards  uint64[E][2W]  words 0..W-1 black discs, W..2W-1 white discs
 *       meta    uint16[E]      bit0 white to move (player_turn == WHITE_DISK)
 *                              bit1 terminated
 *                              bits2-3 winner: 0 NO_DISK / draw, 1 WHITE, 2 BLACK
 *                              bits8-15 random-opening plies still to play
 *       legal   uint64[E][W]   possible_moves -- NOT recomputed on terminal
 *                              plies, exactly like the reference (othello.py:431-433)
 *   - Return value: OTH_OK (0) or a negative OTH_E* code; oth_last_error()
 *     gives the message for the calling thread.
 *   - A handle is bound to one device; calls on one handle must be serialised
 *     by the caller.  Separate handles are independent.
 */
#ifndef OTHELLO_MI355X_H
#define OTHELLO_MI355X_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oth_env oth_env;
typedef void *oth_stream_t; /* hipStream_t */

enum {
    OTH_OK = 0,
    OTH_EINVAL = -1, /* bad argument (board size outside [4,16], NULL pointer, ...) */
    OTH_EHIP = -2,   /* a HIP runtime call failed */
    OTH_ENOMEM = -3
};

/* create flags: the reference's constructor switches (othello.py:222-227) */
enum {
    OTH_SUDDEN_DEATH = 1, /* sudden_death_on_invalid_move */
    OTH_DISK_REWARD = 2,  /* num_disk_as_reward */
    OTH_AUTO_RESET = 4    /* batched only: reset an env right after its terminal ply */
};

/* on-device scripted policies (simple_policies.py): RandomPolicy, GreedyPolicy,
 * MaxiMinPolicy(max_search_depth = d) for d = 1 .. OTH_MAXIMIN_MAX_DEPTH as
 * OTH_POLICY_MAXIMIN(d); MAXIMIN1 plays exactly GREEDY's moves */
enum {
    OTH_POLICY_RANDOM = 0,
    OTH_POLICY_GREEDY = 1,
    OTH_POLICY_MAXIMIN1 = 2,
    OTH_POLICY_MAXIMIN2 = 3,
    OTH_POLICY_MAXIMIN3 = 4
};
#define OTH_MAXIMIN_MAX_DEPTH 10
#define OTH_POLICY_MAXIMIN(d) (OTH_POLICY_MAXIMIN1 + (d) - 1)
#define OTH_POLICY_LAST OTH_POLICY_MAXIMIN(OTH_MAXIMIN_MAX_DEPTH)
/* oth_policy_actions, oth_step_policy and oth_reset_vs / oth_step_vs refuse
 * MaxiMin(d >= 3) calls whose searches are estimated above this many leaves.
 * The first estimate is E x b^d x the searches per board in the call (n_plies
 * for oth_step_policy, 2 opponent replies for the _vs calls) with b = max(2,
 * N*N / 6) moves per position (8x8 middle games: ~10).  Above the budget the
 * call reads the boards (a synchronisation of `stream`; refused during a stream
 * capture) and bounds each live board's search by its own position: its
 * possible_moves at the root, then at most min(b, e - j) moves at level j for
 * e empty squares, since every level places a disc (simple_policies.py:138).
 * So late-game boards search to any depth the budget allows (one 8x8 board
 * with 10 empty squares at depth 10: <= 10! leaves).  Refused calls launch
 * nothing; split the boards over several calls or search shallower. */
#define OTH_MAXIMIN_LEAF_BUDGET 17179869184.0

/* observation layouts */
enum {
    OTH_OBS_BOARD = 0,       /* (E,N,N)   get_observation(): mover +1, opponent -1 (othello.py:363-369) */
    OTH_OBS_BOARD_LEGAL = 1, /* (E,2,N,N) get_observation() with possible_actions_in_obs (othello.py:370-376) */
    OTH_OBS_MAKE_STATE = 2,  /* (E,4,N,N) util.make_state(obs, env) planes (util.py:48-74) */
    OTH_OBS_ABSOLUTE = 3,    /* (E,N,N)   board_state: white +1, black -1 (othello.py:257) */
    OTH_OBS_LEGAL = 4        /* (E,N,N)   possible_moves as 0 / 1 (othello.py:313-343; the plane of
                                          OTH_OBS_BOARD_LEGAL alone: int8 views as a bool mask) */
};
/* observation element types; OTH_BF16 is bfloat16 (the observations' values
 * -1 / 0 / +1 are exact in it): half the bytes of float32 for a network that
 * takes bfloat16 input, e.g. make_state for a learner under bf16 autocast */
enum { OTH_I8 = 0, OTH_I32 = 1, OTH_I64 = 2, OTH_F32 = 3, OTH_F64 = 4, OTH_BF16 = 5 };

/* masked-categorical modes (oth_masked_sample) */
enum {
    OTH_MASKED_SAMPLE = 0, /* FixedCategorical(...).sample() / np.random.choice: actions out */
    OTH_MASKED_MODE = 1,   /* FixedCategorical(...).mode(): first largest legal logit; actions out */
    OTH_MASKED_EVAL = 2,   /* evaluate_actions: actions in, log-probs of those actions out */
    /* or-ed into a mode: entropy[e] = entropy of the UNMASKED categorical over
     * all N*N squares, as Policy.evaluate_actions returns it (dist.entropy(),
     * model.py:175; the caller takes the mean) instead of the masked one */
    OTH_MASKED_FULL_ENTROPY = 4
};

/* OthelloBaseEnv.__init__ (othello.py:222-254) for n_envs boards of size
 * board_size (clamped to >= 4 like othello.py:230; > 16 is OTH_EINVAL).
 * seed / env_id_base key the Philox RNG of the on-device policies: env i uses
 * id env_id_base + i, so a sharded run reproduces an unsharded one.
 * initial_rand_steps: SimpleOthelloEnv's random-opening length bound
 * (othello.py:62-63) applied by oth_reset and auto-reset.  Boards start reset. */
int oth_create(int32_t n_envs, int32_t board_size, uint32_t flags, uint64_t seed, uint32_t env_id_base,
               int32_t initial_rand_steps, int32_t device, oth_env **out);
int oth_destroy(oth_env *env);

/* OthelloBaseEnv.reset (othello.py:265-271) for every env, or only where
 * mask[e] != 0 (mask: device uint8[E] or NULL). */
int oth_reset(oth_env *env, const uint8_t *mask, oth_stream_t stream);

/* OthelloBaseEnv.step (othello.py:412-462) with external actions int32[E].
 * Out: rewards int32[E], dones uint8[E] (either may be NULL).  An env that is
 * already terminated is left unchanged and reports done = 1, reward = 0 (the
 * reference raises ValueError there, othello.py:415-416; the single-env
 * wrapper does so on the host). */
int oth_step(oth_env *env, const int32_t *actions, int32_t *rewards, uint8_t *dones, oth_stream_t stream);

/* oth_step, then the observation of the stepped boards in the same call:
 * OthelloBaseEnv.step's returned get_observation() (othello.py:462; layout
 * OTH_OBS_BOARD / OTH_OBS_BOARD_LEGAL) or any oth_observe layout / dtype into
 * obs (E, planes, N, N).  The values are exactly oth_step followed by
 * oth_observe: the state after the ply (and after an auto-reset).  One launch
 * where the board is one word and N*N % 4 == 0 with obs aligned to 4
 * elements (the observation is written from the registers that stepped the
 * board, nothing read back); two launches otherwise. */
int oth_step_observe(oth_env *env, const int32_t *actions, int32_t *rewards, uint8_t *dones, int32_t layout,
                     int32_t dtype, void *obs, oth_stream_t stream);

/* n_plies plies of on-device play: each env's mover picks with `policy`
 * (RandomPolicy.get_action simple_policies.py:37-41 / GreedyPolicy.get_action
 * :69-92, or a random move while random-opening plies remain) and steps.
 * Outputs are [n_plies][E] (any may be NULL): the action played (-1 for an
 * env that was already terminated), reward, done.  Finished games are tallied
 * into the handle's win/draw/loss counters (oth_counts). */
int oth_step_policy(oth_env *env, int32_t policy, int32_t n_plies, int32_t *actions, int32_t *rewards,
                    uint8_t *dones, oth_stream_t stream);

/* OthelloEnv (othello.py:96-214) for every env: the protagonist's colour per
 * env (protagonist: device int8[E] of +1 white / -1 black, NULL = all white,
 * the reference default) and an embedded opponent played on the device
 * (OTH_POLICY_RANDOM / OTH_POLICY_GREEDY).
 *   oth_reset_vs: OthelloEnv.reset (:151-174) -- reset, then the opponent
 *     replies (with its policy) until the protagonist is to move.
 *   oth_step_vs:  OthelloEnv.step (:176-200) -- the protagonist plays
 *     actions[e] (a random move while random-opening plies remain), then the
 *     opponent replies until the protagonist is to move again or the game
 *     ends.  rewards[e] is the protagonist's step reward, negated when an
 *     opponent ply ended the game (:200); plies[e] (may be NULL) counts the
 *     plies applied.  With OTH_AUTO_RESET a finished env is reset_vs'd.
 * Random draws: the j-th ply of call number c (the handle's ply counter,
 * advanced by one per call) uses Philox block (c*256 + j) / 4, word (c*256 + j) % 4. */
int oth_reset_vs(oth_env *env, int32_t opponent_policy, const int8_t *protagonist, const uint8_t *mask,
                 oth_stream_t stream);
int oth_step_vs(oth_env *env, int32_t opponent_policy, const int32_t *actions, const int8_t *protagonist,
                int32_t *rewards, uint8_t *dones, int32_t *plies, oth_stream_t stream);
/* oth_step_vs, then the observation (layout / dtype as oth_observe) of the
 * boards as the call leaves them -- OthelloEnv.step's returned obs
 * (othello.py:200) with OTH_OBS_BOARD -- into obs in the same call: one launch
 * for one-word boards against a random or greedy opponent with obs aligned to 4
 * elements, else two. */
int oth_step_vs_observe(oth_env *env, int32_t opponent_policy, const int32_t *actions, const int8_t *protagonist,
                        int32_t *rewards, uint8_t *dones, int32_t *plies, int32_t layout, int32_t dtype, void *obs,
                        oth_stream_t stream);

/* possible_moves of every env as masks uint64[E][W] (othello.py:242, :270, :466). */
int oth_legal(oth_env *env, uint64_t *out, oth_stream_t stream);

/* get_possible_actions(board) (othello.py:313-343), stateless: n canonical
 * boards given as mover / opponent masks uint64[n][W] -> uint64[n][W]. */
int oth_legal_moves(int32_t board_size, int32_t n, const uint64_t *mover, const uint64_t *opp, uint64_t *out,
                    oth_stream_t stream);

/* GreedyPolicy.get_action (simple_policies.py:69-92) for the side to move in
 * every env: argmax over possible_moves of the discs flipped, lowest square
 * on ties; -1 where possible_moves is empty.  Out int32[E]. */
int oth_greedy_actions(oth_env *env, int32_t *out, oth_stream_t stream);

/* The move of a deterministic scripted policy (OTH_POLICY_GREEDY or
 * OTH_POLICY_MAXIMIN(d): MaxiMinPolicy(d).get_action, simple_policies.py:157-163)
 * for the side to move in every env; -1 where possible_moves is empty.
 * MaxiMin(d >= 3) searches each board with a whole wave (the root's moves and
 * their replies spread over the lanes); above OTH_MAXIMIN_LEAF_BUDGET estimated
 * leaves (position-aware, see there) the call is refused (OTH_EINVAL) before
 * anything is launched. */
int oth_policy_actions(oth_env *env, int32_t policy, int32_t *out, oth_stream_t stream);

/* Observations: layout OTH_OBS_*, dtype OTH_I8..OTH_F64, out (E, planes, N, N). */
int oth_observe(oth_env *env, int32_t layout, int32_t dtype, void *out, oth_stream_t stream);

/* Copy the state out / in (exchange format above).  In oth_set_state any of
 * the three sources may be NULL (left unchanged): set_board_state
 * (othello.py:380-389) replaces only the boards. */
int oth_get_state(oth_env *env, uint64_t *boards, uint16_t *meta, uint64_t *legal, oth_stream_t stream);
int oth_set_state(oth_env *env, const uint64_t *boards, const uint16_t *meta, const uint64_t *legal,
                  oth_stream_t stream);

/* set_player_turn (othello.py:464-466): turn (+1 white / -1 black) for every
 * env (or where mask[e] != 0), then recompute possible_moves. */
int oth_set_player_turn(oth_env *env, int32_t turn, const uint8_t *mask, oth_stream_t stream);

/* count_disks (othello.py:468-471): out int32[E][2] = (white_cnt, black_cnt). */
int oth_count_disks(oth_env *env, int32_t *out, oth_stream_t stream);

/* Win/draw/loss tally of games finished by oth_step / oth_step_policy since
 * the last reset of the counters: out int64[3] = {black wins, draws, white
 * wins} (device pointer).  reset != 0 zeroes the counters after the copy. */
int oth_counts(oth_env *env, int64_t *out, int32_t reset, oth_stream_t stream);

/* The harnesses' tally (run.py:100-130, the README's wins / draws / loses) of
 * games finished by oth_step_vs, from each board's protagonist's side: out
 * int64[3] = {protagonist wins, draws, protagonist losses} (device pointer);
 * reset != 0 zeroes the counters after the copy. */
int oth_counts_vs(oth_env *env, int64_t *out, int32_t reset, oth_stream_t stream);

/* Masked categorical over each board's legal squares (policy head of the
 * learners; replaces the per-sample loops of
 * pytorch_a2c_ppo_acktr_gail/a2c_ppo_acktr/model.py:60-99 Policy.act,
 * model.py:156-178 Policy.evaluate_actions and ppo.py:228-298 PPO.get_action).
 * n boards: logits float32 rows of N*N with row stride ld (elements), legal
 * uint64[n][W] (e.g. oth_legal's output), device pointers.
 *   OTH_MASKED_SAMPLE: action = the first legal square whose cumulative
 *     softmax mass exceeds u * total, u = uniforms[e] in [0,1) if uniforms is
 *     non-NULL, else a Philox draw keyed (seed, id_base + e, counter);
 *   OTH_MASKED_MODE: action = the lowest legal square of the largest logit;
 *   OTH_MASKED_EVAL: actions is an INPUT.
 * log_probs[e] = log softmax over the legal squares at the action (0 when the
 * board has no legal move or the action is not one of them, model.py:69-71,
 * :165); entropy[e] = entropy of the masked distribution (0 with no legal
 * move).  A board without legal moves samples action 0 (model.py:69-71).
 * log_probs / entropy may be NULL.  Logits must be finite. */
int oth_masked_sample(int32_t board_size, int32_t n, const float *logits, int64_t ld, const uint64_t *legal,
                      const float *uniforms, uint64_t seed, uint32_t id_base, uint64_t counter, int32_t mode,
                      int32_t *actions, float *log_probs, float *entropy, oth_stream_t stream);

/* oth_masked_sample over the handle's own boards and possible_moves, keyed
 * by the handle's seed and env ids. */
int oth_sample_actions(oth_env *env, const float *logits, int64_t ld, const float *uniforms, uint64_t counter,
                       int32_t mode, int32_t *actions, float *log_probs, float *entropy, oth_stream_t stream);

/* One ply of the learners' loop in one launch: oth_sample_actions (mode
 * OTH_MASKED_SAMPLE or OTH_MASKED_MODE, optionally | OTH_MASKED_FULL_ENTROPY)
 * over the handle's possible_moves, then oth_step with the chosen actions
 * (Policy.act model.py:60-99 / PPO.get_action ppo.py:228-262, then
 * OthelloBaseEnv.step othello.py:412-462).  Results are bit-identical to the
 * two calls.  Out: actions int32[E] (required), log_probs / entropy float[E],
 * rewards int32[E], dones uint8[E] (each may be NULL).  Advances the ply
 * counter by one; `counter` is the sample counter as in oth_sample_actions. */
int oth_sample_step(oth_env *env, const float *logits, int64_t ld, const float *uniforms, uint64_t counter,
                    int32_t mode, int32_t *actions, float *log_probs, float *entropy, int32_t *rewards,
                    uint8_t *dones, oth_stream_t stream);

/* oth_sample_step, then the observation of the stepped boards (layout, dtype
 * as oth_observe: e.g. OTH_OBS_MAKE_STATE in OTH_F32, the learners' next input,
 * util.py:48-74) into obs in the same call: bit-identical to oth_sample_step +
 * oth_observe.  One launch for N*N % 4 == 0 with obs aligned to 4 elements. */
int oth_sample_step_observe(oth_env *env, const float *logits, int64_t ld, const float *uniforms, uint64_t counter,
                            int32_t mode, int32_t *actions, float *log_probs, float *entropy, int32_t *rewards,
                            uint8_t *dones, int32_t layout, int32_t dtype, void *obs, oth_stream_t stream);

/* One board's state in the reference's terms, as the single-board drop-in
 * classes (OthelloBaseEnv / SimpleOthelloEnv / OthelloEnv, othello.py:21-501;
 * BASELINE config 1) return it after every call.  W used words per colour. */
#define OTH_RECORD_MAX_WORDS 4
#define OTH_RECORD_GREEDY 2       /* oth_step_sync's `step` bit: also compute the record's greedy move */
#define OTH_RECORD_NO_GREEDY (-2) /* the record's greedy field when that bit was not given */
#define OTH_RECORD_MAX_SQUARES 256
typedef struct oth_record {
    uint64_t black[OTH_RECORD_MAX_WORDS]; /* the board (exchange format) */
    uint64_t white[OTH_RECORD_MAX_WORDS];
    uint64_t legal[OTH_RECORD_MAX_WORDS]; /* possible_moves (stale on terminal plies, as the reference's) */
    uint32_t seq;                         /* the call's sequence number (written last) */
    uint16_t meta;                        /* exchange-format meta: player_turn, terminated, winner */
    uint8_t done;                         /* the step's done (0 without a step) */
    uint8_t planes;                       /* observation planes in obs: 1, or 2 with the legal plane */
    int32_t reward;                       /* the step's reward (0 without a step) */
    int32_t white_cnt, black_cnt;         /* count_disks (othello.py:468-471) */
    int32_t greedy;                       /* GreedyPolicy.get_action for the side to move (simple_policies.py:69-92);
                                             -1 without a possible move; OTH_RECORD_NO_GREEDY unless the call
                                             asked for it (OTH_RECORD_GREEDY) */
    int8_t obs[2 * OTH_RECORD_MAX_SQUARES];   /* get_observation() (othello.py:363-378): planes x N x N */
    int8_t board_state[OTH_RECORD_MAX_SQUARES]; /* board_state (othello.py:257): white +1, black -1 */
} oth_record;

/* The single-board drop-in path in one launch and one wait: if step & 1,
 * OthelloBaseEnv.step (othello.py:412-462) of board `board` with the host value
 * `action` (any int: not in possible_moves takes the invalid path; a
 * terminated board is left as it is and reports done, as oth_step), then the
 * board's record (layout OTH_OBS_BOARD or OTH_OBS_BOARD_LEGAL for obs) is
 * written by the same kernel into a mapped host buffer the handle owns, and the
 * call returns once it has landed: *out points at it until the next call on
 * this handle.  step & 1 == 0 only records (after reset / set_state /
 * set_player_turn).  step & OTH_RECORD_GREEDY also computes GreedyPolicy's move
 * for the side to move (one lane's bit-plane flip counts: about 0.5 us of the
 * call, so only when a greedy policy reads the record). */
int oth_step_sync(oth_env *env, int32_t board, int32_t step, int32_t action, int32_t layout,
                  const oth_record **out, oth_stream_t stream);

/* Global ply counter of the handle: the Philox counter of the next eager ply
 * (random policy, openings, device opponents).  Host value only; setting it
 * does not touch graph regions' counter ranges (below). */
uint64_t oth_ply_counter(const oth_env *env);
int oth_set_ply_counter(oth_env *env, uint64_t ply);

/* HIP-graph regions (no reference counterpart: the reference has no device).
 * Every entry point only enqueues kernels on `stream`, so a region of calls can
 * be captured and replayed.  The Philox counters a capture bakes in are host
 * values; to make every replay draw fresh numbers without reusing any counter
 * of eager calls or of other graphs, each region owns a disjoint counter range:
 *   oth_graph_begin: opens region k (k = 1 .. OTH_GRAPH_SLOTS-1, *slot = k);
 *     until oth_graph_end the handle's ply counter runs from
 *     k << OTH_GRAPH_COUNTER_SHIFT and launches add the device offsets of slot k;
 *   oth_graph_end: closes it, restores the eager ply counter, *d_ply = plies
 *     the region consumed; if enqueue != 0 it enqueues (as the region's last
 *     node) the advance of slot k's offsets by (d_ply, d_sample), so replay r
 *     draws the counters (k << SHIFT) + r * d + j.  d_sample is what the caller's
 *     sample counter (oth_sample_actions) consumed inside the region, whose
 *     range must start at k << SHIFT as well.
 *   oth_graph_offsets: slot k's (ply, sample) offsets; synchronises the device
 *     (never call it while a capture is active).
 *   oth_graph_release: gives slot k back (its graph is dropped, or its capture
 *     failed); oth_graph_begin hands out the lowest free slot.  The slot's
 *     offsets are kept, so a later region on it still draws fresh counters.
 * Eager launches use slot 0, always 0. */
#define OTH_GRAPH_SLOTS 64
#define OTH_GRAPH_COUNTER_SHIFT 40
int oth_graph_begin(oth_env *env, int32_t *slot);
int oth_graph_end(oth_env *env, uint64_t d_sample, int32_t enqueue, uint64_t *d_ply, oth_stream_t stream);
int oth_graph_offsets(const oth_env *env, int32_t slot, uint64_t out[2]);
int oth_graph_release(oth_env *env, int32_t slot);

/* Handle geometry: n_envs, board_size, W. */
int oth_shape(const oth_env *env, int32_t *n_envs, int32_t *board_size, int32_t *words);

/* Message of the last failing call on this thread ("" if none). */
const char *oth_last_error(void);

/* Library version string. */
const char *oth_version(void);

#ifdef __cplusplus
}
#endif
#endif /* OTHELLO_MI355X_H */
