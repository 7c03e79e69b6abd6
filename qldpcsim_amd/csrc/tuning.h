// tuning.h — compile-time knobs of the HIP kernels, all in one place.
//
// The shipping build uses the measured defaults below (DESIGN.md cites the
// A/B that chose each). Experiment builds (tools/build_variants.sh) may set
// any of them with -D, but only together with -DQLDPC_EXPERIMENTS: a knob
// defined without it is a build error, so no ablation or diagnostic setting
// reaches the product library by accident. Runtime kernel-family choices are
// library options (qldpc_set_option, include/qldpc_decoder.h), not knobs.
#pragma once

#if !defined(QLDPC_EXPERIMENTS) &&                                                                   \
    (defined(QLDPC_ABLATE) || defined(QLDPC_ABLATE_L) || defined(QLDPC_ABLATE_OSD) ||               \
     defined(QLDPC_OSD_TIMING) || defined(QLDPC_VN_PAIR) || defined(QLDPC_FLOOD_WPE) ||             \
     defined(QLDPC_VN_H) || defined(QLDPC_HBM_WAVES) || defined(QLDPC_HBM_UC) ||                    \
     defined(QLDPC_OSD_WPE) || defined(QLDPC_OSD_PRIO) || defined(QLDPC_ABLATE_ORD) ||               \
     defined(QLDPC_OSD_DSPLIT) || defined(QLDPC_MSL_GT) || defined(QLDPC_OSD_PAIRS) ||               \
     defined(QLDPC_MSL_KARGS) || defined(QLDPC_BP_SAT) || defined(QLDPC_BP_VNPRIO) ||                \
     defined(QLDPC_BP_CNPRIO) || defined(QLDPC_BP_LHPRIO) || defined(QLDPC_BP_FCNPRIO) ||            \
     defined(QLDPC_MSL_PRIO))
#error "kernel tuning knobs are for experiment builds: add -DQLDPC_EXPERIMENTS"
#endif

// knock-outs for timing attribution (experiment builds only)
#ifndef QLDPC_ABLATE
#define QLDPC_ABLATE 0       // flooding decode_kernel: 1 = skip VN, 2 = skip CN
#endif
#ifndef QLDPC_ABLATE_L
#define QLDPC_ABLATE_L 0     // ms_layered_kernel: bit 0 skips CN, bit 1 VN, bit 2 the filter
#endif
#ifndef QLDPC_ABLATE_OSD
#define QLDPC_ABLATE_OSD 0   // osd_block_kernel: bit 0 skips phase D, bit 1 the engine
#endif
#ifndef QLDPC_ABLATE_ORD
#define QLDPC_ABLATE_ORD 0   // osd_order_kernel: bit 0 skips the <= 256-key networks, bit 1 the partitions
#endif
#ifndef QLDPC_OSD_TIMING
#define QLDPC_OSD_TIMING 0   // osd_block_kernel sums per-phase cycles into OsdArgs::prof (option osd_prof)
#endif

// measured defaults
#ifndef QLDPC_VN_PAIR
#define QLDPC_VN_PAIR 1      // ms_flood_kernel VN: two 64-variable chunks per trip
#endif
#ifndef QLDPC_FLOOD_WPE
#define QLDPC_FLOOD_WPE 3    // ms_flood_kernel: waves per SIMD the register budget targets (KC <= 4)
#endif
#ifndef QLDPC_VN_H
#define QLDPC_VN_H 4         // ms_layered_kernel: variables per lane on layers of > 128 adjacent variables
#endif
#ifndef QLDPC_HBM_WAVES
#define QLDPC_HBM_WAVES 4    // hbm_tile_kernel: waves per 64-slot tile (kernel names spell out 4)
#endif
#ifndef QLDPC_HBM_UC
#define QLDPC_HBM_UC 1       // hbm_tile_kernel: checks per load step (1: 16 waves per CU; 2, 4 slower)
#endif
#ifndef QLDPC_OSD_WPE
#define QLDPC_OSD_WPE 4      // osd_block_kernel, two rows per thread: waves per SIMD (3: no spills, slower)
#endif
#ifndef QLDPC_OSD_PRIO
#define QLDPC_OSD_PRIO 3     // osd_block_kernel: s_setprio of the engine wave during phase B (0: none;
                             // 1 and 3 both -3.3 % per launch, profiles/r04am/)
#endif
#ifndef QLDPC_OSD_DSPLIT
#define QLDPC_OSD_DSPLIT 12  // osd_block_kernel phase D: pivot-row words read in two batches when more
                             // than this many remain (0: one batch); 12: 93 -> 16 spilled VGPRs,
                             // 26.85 -> 26.56 ms per 68,301 shots (profiles/r05/osd_dsplit_ab.jsonl)
#endif
#ifndef QLDPC_OSD_PAIRS
#define QLDPC_OSD_PAIRS 1    // osd_block_kernel phase D: this block's pivots applied two at a time from
                             // a table of pair XORs (one LDS row read per nonzero bit pair): 22.82 ->
                             // 22.38 ms per 68,301 shots (profiles/r05/osd_pairs_ab.jsonl)
#endif
#ifndef QLDPC_MSL_KARGS
#define QLDPC_MSL_KARGS 1    // ms_layered_kernel: arguments used only outside the layer loops reloaded
                             // from the kernarg segment at their use (125 -> 16 spilled SGPRs; LP118_2
                             // p = 0.1 35.78 -> 35.07 ms per launch, profiles/r05/msl_kargs_ab.json)
#endif
#ifndef QLDPC_MSL_GT
#define QLDPC_MSL_GT 1       // ms_layered_kernel<DC, 1>: row table and filter words in global memory, 8
                             // waves per CU (1: LP118_2 p = 0.1 39.9 -> 36.5 ms per launch), or in LDS (0)
#endif
#ifndef QLDPC_BP_SAT
#define QLDPC_BP_SAT 1       // layered BP check node: a wave whose every edge has |v2c / 2| >= 19.5
                             // (NumPy's tanh = +-1 exactly) takes c2v = +-2 atanh(1 - eps) without the
                             // tanh, the product, the division and the atanh (0: always the full path);
                             // LP118_2 p = 0.1 111.8 -> 107.6 ms per launch (profiles/r05/bp_sat_ab.json)
#endif
#ifndef QLDPC_BP_VNPRIO
#define QLDPC_BP_VNPRIO 2    // bp_team_lg_kernel: s_setprio of a layer's variable-node phase (0: none);
                             // 2: LP118_2 p = 0.1 107.2 -> 103.8 ms per launch (the check-node phase at
                             // priority 2 instead: 106.3 ms), profiles/r05/bp_prio_ab.json; levels 1 / 3
                             // within 0.7 % of 2 (bp_prio_levels_ab.json)
#endif
#ifndef QLDPC_BP_CNPRIO
#define QLDPC_BP_CNPRIO 2    // layered BP check nodes at priority 1 from entry to the tanh (1), to the
                             // division (2), or from the division to the store (3); 0: none. LP118_2
                             // p = 0.1 103.9 ms per launch -> 103.3 / 102.1 / 106.5 (bp_cnprio_ab.json)
#endif
#ifndef QLDPC_BP_FCNPRIO
#define QLDPC_BP_FCNPRIO 2   // the same modes for the flooding BP kernel's check nodes; 2: LP118_0 BP-F
                             // fixed work 76.9 -> 73.4 ms per launch (profiles/r05/prio_msl_bpf_ab.json;
                             // 78.5 -> 76.7 on a slower box, round5_ab_start_vs_head.json); mode 1: +1.6 %,
                             // with the flooding VN at 2 as well: within noise (bpf_prio_modes_ab.json)
#endif
#ifndef QLDPC_MSL_PRIO
#define QLDPC_MSL_PRIO 1     // ms_layered_kernel: check nodes at priority 1 (1) or variable nodes at 1 (2);
                             // LP118_2 p = 0.1 35.05 -> 34.84 / 35.58 ms per launch (prio_msl_bpf_ab.json)
#endif
#ifndef QLDPC_BP_LHPRIO
#define QLDPC_BP_LHPRIO 1    // bp_team_lg_kernel: priority of the layer head (stop test, prefetch issue);
                             // 1: 102.1 -> 101.4 ms per LP118_2 p = 0.1 launch (bp_lhprio_ab.json); 2, or
                             // 3 with the VN at 3: within 0.1 % (bp_lhprio_levels_ab.json)
#endif

// Variants measured and not kept (their A/B records stay under profiles/r05/,
// DESIGN.md §3): batched fold permutes (bp_fold_ab.json), unmasked BP
// prefetches (bp_uload_ab.json), the saturated-check shortcut in flooding BP,
// flooding-BP VN priority (bpf_prio_modes_ab.json), OSD phase-A priority
// (osd_aprio_ab.jsonl), exact free-slot counts in the OSD engine, the layered
// VN's layer-head adjacency reads (msl_vn_knobs_ab.json). Their code paths
// were removed in round 6.
