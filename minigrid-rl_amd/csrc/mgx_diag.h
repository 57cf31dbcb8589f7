// mgx_diag.h -- every diagnostic and A/B switch of the engine, in one place.
//
// The product build (`make -C minigrid-rl_amd`, __graft_entry__.build()) defines none of them and the
// product library reads no environment variable: its scheduling is fixed at compile time.  Each switch
// is a build of its own, loaded instead of libmgx.so through MGX_LIB_PATH (mgx/_lib.py), e.g.
//
//   make -C minigrid-rl_amd EXTRA="-DMGX_RSTAMPS=1" OUT=mgx/libmgx_rstamps.so
//   MGX_LIB_PATH=$PWD/minigrid-rl_amd/mgx/libmgx_rstamps.so python tools/diag_rollout_phases.py
//
// Clocks are s_memtime cycles summed into the device counters (mgx_debug_counters).
#pragma once

// ---- clocks ------------------------------------------------------------------------------------
#ifndef MGX_STAMPS          // mgx_step_kernel phase clocks -> counters[4..7] (1, 2, 3: phase groupings)
#define MGX_STAMPS 0
#endif
#ifndef MGX_RSTAMPS         // mgx_rollout_kernel: wave 0's clocks per phase, summed over the steps -> counters[4..7]
#define MGX_RSTAMPS 0
#endif
#ifndef MGX_REFILL_CLOCK    // refill wave clocks, attempt rounds (busiest lane) and a histogram -> counters[8..29]
#define MGX_REFILL_CLOCK 0
#endif
#ifndef MGX_GEN_STAMPS      // generator section clocks (1: + iteration counts, 2: clocks only).  They inflate the
#define MGX_GEN_STAMPS 0    // wave's time ~5x (a global atomic per stamp): elimination (MGX_GEN_SKIP) is the measure
#endif

// ---- elimination builds: the outputs are then NOT the reference's -------------------------------
#ifndef MGX_GEN_SKIP        // skip generator sections: 1 keys + objects, 2 door positions, 4 goal + agent,
#define MGX_GEN_SKIP 0      // 8 walls + door draws; inside the keys + objects loop 32 the object choice draw;
                            // 64 the refill's mission-token copy into the ring header (SB3 layout's tokens)
#endif
#ifndef MGX_GEN_PREFIX2      // run every MT-only prefix draw sequence (mission / room count, door colours, door positions)
#define MGX_GEN_PREFIX2 0    // twice, the first discarded: an upper bound of what memoising the prefix could save (round 6)
#endif
#ifndef MGX_PFX_MEMO         // 1: multi-room refills look the MT-only generator prefix up in per-position records
#define MGX_PFX_MEMO 1       // (KParams.pfx, round 6); 0: drawn in every attempt (A/B)
#endif
#ifndef MGX_DIAG_SKIP       // mgx_step_kernel: skip store classes (2 stack roll, 4 missions, 16 grids)
#define MGX_DIAG_SKIP 0
#endif

// ---- A/B variants of product choices (the defaults ARE the product) ----------------------------
// Retired in round 5 (settled, compiled in as the product's choice): NT_STACK 0, SYNC_FULL 0, MT_TOPUP 0,
// STEP_S8 1, ROLL_DEFER_ROWS 1, ROLL_POPCNT 1, ROLL_S8 1, REFILL_S8 1, ROLLOUT_FIRST 0, STEP_PRIO 0,
// REFILL_GENERIC 0, REFILL_MEAN 2, REFILL_ROUNDS 2 (their measurements: DESIGN.md §4-5).
#ifndef MGX_MT_WG1          // MT window groups per refill lane at S <= 8 (8 or 16; 16 for larger grids)
#define MGX_MT_WG1 8
#endif
#ifndef MGX_ROLL_VMKEEP      // fused rollout's two per-step barriers: -1 __syncthreads (waits for every store),
#define MGX_ROLL_VMKEEP 8   // N >= 0: LDS complete, <= N vector-memory ops of the wave in flight, s_barrier
#endif                      // (round 4 A/B: default line +8-10 % at 8 or 12, 20-step line within noise)
#ifndef MGX_REFILL_EPW       // envs per S = 8 refill wave: 0 auto (32 when 64-env waves leave SIMDs idle), 16, 32, 64
#define MGX_REFILL_EPW 0
#endif
#ifndef MGX_ROLL_EPB_S16     // envs per fused-rollout block at S = 16 (config 5): 64, or 32 (twice the blocks, half the LDS;
#define MGX_ROLL_EPB_S16 32  // round 5 A/B, 2 rotating rounds: config 5 5.13-5.16 vs 5.05-5.06 x 10^9, kernel 24.4-24.6 vs
#endif                      // 24.9 us per step)
#ifndef MGX_ROLL_LOGIC_PRIO  // fused rollout: s_setprio of wave 0 during its step logic (0: none; the block waits for it).
#define MGX_ROLL_LOGIC_PRIO 3  // Round 6 A/B (3 rotating rounds, prefix records in: refill and rollout balanced): driver's line
#endif                        // 6.76-7.01 vs 6.70-6.83 x 10^9, default line 9.23 vs 8.46, config 4 6.03 vs 6.16 (round 5: neutral)
#ifndef MGX_SLIDE_FENCE      // 1: the MT slide orders its reductions with __threadfence() (an L2 write-back per workgroup),
#define MGX_SLIDE_FENCE 1    // 0: by waiting for its returning atomics.  Round 5 A/B (rotating order, 3 + 2 rounds): the
#endif                      // fenced slide is the faster pipeline -- 20-step line 5.88 vs 5.71, default line 7.97-8.07 vs 7.35
                            // x 10^9 (its write-back also cleans the L2 the next refill works in); kept
#ifndef MGX_STEP_LOGIC_PRIO  // per-step kernel: s_setprio of wave 0 during its step logic (0: none).  Round 5 A/B (3
#define MGX_STEP_LOGIC_PRIO 3  // rotating rounds, compact layout, 256 steps): 5.64-5.70 vs 5.46-5.47 x 10^9, kernel 7.6-7.7
#endif                        // vs 8.1 us per step (the refill beside it 510 vs 450 us per epoch: it no longer bounds)
#ifndef MGX_PUBN_ACQUIRE     // 1: the fused rollout reads ring_pubn with an agent-scope acquire (0: relaxed; A/B of the
#define MGX_PUBN_ACQUIRE 1   // acquire's cost)
#endif
#ifndef MGX_NT_REC           // 1: the refill writes its ring records with non-temporal (streaming) stores (round 6 A/B)
#define MGX_NT_REC 0
#endif
#ifndef MGX_NT_ROWS          // 1: the fused rollout copies its observation rows out with non-temporal stores (round 6 A/B)
#define MGX_NT_ROWS 0
#endif
#ifndef MGX_ROLL_LDS_PAD     // diagnostic: extra dynamic LDS bytes per fused-rollout workgroup (fewer workgroups per CU:
#define MGX_ROLL_LDS_PAD 0   // the residency's share of the rollout's time, round 6)
#endif
#ifndef MGX_SERIAL_REFILL   // refill on the caller's stream (the refill alone, for timing it)
#define MGX_SERIAL_REFILL 0
#endif
#ifndef MGX_REFILL_PRIO     // s_setprio of the refill's waves over co-resident step / rollout waves (0..3)
#define MGX_REFILL_PRIO 2
#endif
