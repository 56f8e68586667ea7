// C ABI over the MI355X validation kernels (K1 GEMM, K2 HBM stream,
// K3 fill/reference/verify). Built for gfx950 only into
//   nvidia_terraform_modules_amd/ops/libntm_validation.so   (Python, ctypes)
//   validation/build/amdgpu-validate                        (Job entrypoint)
// Every entry point is stream-ordered, allocation-free and sync-free, so it
// can be captured in a hipGraph (playbook §6 Guideline 9).
//
// Only the kernels the default dispatch can select are instantiated here
// (pingpong8c / pingpong8b 256x256, the six tile shapes and split-K, K1-fp8 on
// the 256x256 kernel and the wave-specialised tiles, K2, K3).
// The non-default K1 builds, schedule knobs and diagnostics live in
// ntm_experimental.hip -> libntm_experimental.so (tests and tools only).
#include "ntm/aux_kernels.hpp"
#include "ntm/gemm_bf16_pp2.hpp"
#include "ntm/gemm_bf16_pp3.hpp"
#include "ntm/gemm_bf16_pp3h.hpp"
#include "ntm/gemm_bf16_pp6.hpp"
#include "ntm/gemm_bf16_sk.hpp"
#include "ntm/gemm_bf16_skh.hpp"
#include "ntm/gemm_bf16_t128.hpp"
#include "ntm/gemm_fp8.hpp"
#include "ntm/gemm_w4k.hpp"

#define NTM_API extern "C" __attribute__((visibility("default")))

namespace {
inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }
inline unsigned stream_grid(size_t work_items, unsigned block) {
  // memory-bound: min(work / block, 256 CUs x 8 blocks)
  size_t g = (work_items + block - 1) / block;
  if (g > 2048) g = 2048;
  if (g == 0) g = 1;
  return (unsigned)g;
}
}  // namespace

NTM_API const char* ntm_version() { return "ntm-validation 0.1.0 gfx950"; }

NTM_API int ntm_gemm_shape_ok(int M, int N, int K) {
  return ntm::gemm::shape_ok(M, N, K) ? 1 : 0;
}

// K1 variants in this (shipping) library: 4 = pingpong8b, the 8-wave 256x256
// kernel with the balanced 8/4/8/4 LDS read schedule (gemm_bf16_pp2.hpp; K %
// 64); 5 = pingpong8c, the same schedule with parity-alternating B buffers, a
// uniform tail-free K loop and the LDS-staged nontemporal epilogue
// (gemm_bf16_pp3.hpp; K % 128); 15 / 16 / 17 / 23 / 24 / 18 = 128x128 /
// 256x128 / 160x160 / 160x128 / 128x160 / 256x160 tiles (gemm_bf16_t128.hpp):
// all but the last on the wave-specialised 8-wave kernel (masked: any M, N % 4,
// K % 8), 256x160 on the 4-wave one (whole tiles, K % 128; its accumulators +
// one fragment set do not fit 256 registers at two waves per SIMD).
// 0 = default: the plan below. Variants 1-3 and 6-14 (the first ping-pong,
// the 4-wave 128x128-per-wave kernel, the persistent kernel, the 32-MFMA
// segment schedules, epilogue knobs) are experimental: libntm_experimental.so.
// Measured on MI355X (tools/gemm_check.py, random bf16, median of 7 rounds,
// profiles/r1_pp3/): 8192^3: 5 1567 TF, 4 1530; 4096^3: 5 1479, 4 1435; then
// variant 5 without s_setprio +1.3-1.7 % (profiles/r1_pp3_knobs) and with the
// LDS-staged epilogue (profiles/r1_epilogue, r1_round7): 8192^3 1623-1635 TF
// vs hipBLASLt 1632-1648, 4096^3 1536 vs 1532-1544 (same processes).
// Variants 4 and 5 pass tools/race_screen.py (bitwise-stable under HBM noise).
// Default: 5 when K % 128 == 0, else 4 (both need K % 64 == 0, K >= 128).
// 25 = pingpong8o, the persistent build of 5 whose C stores overlap the next
// tile's K loop (gemm_bf16_pp6.hpp): the plan runs it in place of 5 when the
// 256x256 part has more tiles than CUs (a CU then crosses a tile boundary) and
// K >= 256. Measured in one process against 5 (tools/gemm_check.py, medians of
// 13 rounds, profiles/r3_k1o/): 8192^3 1634 vs 1622 TF/s (+0.8 %), 5120^3
// 1394 vs 1374 (+1.5 %), 8192x8192x6144 1611 vs 1590 (+1.3 %).
constexpr int kDefaultVariant = 5;
constexpr int kPersistentVariant = 25;
// Boundary stores of the shipping build spread over the 7 phases the quadrants
// allow (gemm_bf16_pp6.hpp SPREAD, "pingpong8od"), round 4: median over 3
// boxes vs hipBLASLt 8192^3 0.998 (plain 0.996), 8192x8192x4096 1.008
// (0.992), 5120^3 1.022 (1.009), 8192x8192x6144 1.005 (0.998); never below
// the plain build on any box (profiles/r4_ab/). Bitwise equal; race screen
// clean (profiles/r4_race/).
constexpr bool kPp6Spread = true;
// K1-fp8 runs the persistent overlap kernel with f8f6f4 MFMAs on VGPR
// accumulators (gemm_bf16_pp6.hpp F8, experimental fp8 knob 30 until round 4)
// on whole 256x256 tiles, one round or more: +0.8 to +3.0 % over the fp8
// pingpong8c at 4096^3, 8192^3, 8192x8192x4096, 8192x4096x8192 and
// 4096x8192x8192 on each of 3 boxes (profiles/r4_fp8/, r4_ab/); bitwise equal.
// With the spread boundary stores too (kPp6Spread; fp8 knob 31): another +1.3
// to +2.0 % at 8192^3 and +2.6 to +4.4 % at 8192x8192x4096 over knob 30 on
// each of 3 boxes (profiles/r4_ab/fp8_spread_*), never below it.
constexpr bool kFp8Persistent = true;
// pingpong8om (variant 47, the persistent overlap kernel on ragged C) measured
// no better than pingpong8cm under the plan (round 4, profiles/r4_om/), so the
// plan never runs it; it lives in libntm_experimental.so (round 5 hygiene).

// Tile-shape plan of the default dispatch: the smallest predicted time
// rounds(tiles) x tile_area / efficiency over 256 CUs, where the efficiencies
// are each kernel's full-chip rate relative to the 256x256 kernel. The plan
// may split C by rows: the top rows on the 256x256 kernel in whole rounds, the
// rest in a second launch on a small tile, so a partial last round of big
// tiles becomes a full round of small ones (6144^3: 3 rounds of 256x256 ->
// 2 rounds + one of 256x128). Alone it picks 128x128 at 2048^3, 160x160 at
// 2560^3 and 3200^3, 256x128 at 2816^3 and 4096x2048x4096, and 256x256 at
// 3072^3, 4096^3 and 8192^3.
// Efficiencies (round 2, wave-specialised 128x128 / 256x128 / 160x160):
// 0.60 / 0.78 at 8192^3 (989 / 1306 vs 1654 TF/s, profiles/r2_ws/policy_ws1.log,
// interleaved in one process); 160x160 at its full-chip rate at 5120^3 (4 full
// rounds). 256x160 (4-wave) is priced from a full round of it against one of
// 256x256 at 4096x2560x4096 (1121 vs 1146 TF/s, r1_t160/policy_plan.log), not
// from its 8192x5120 rate (0.72): at 0.72 the plan split 5120^3 and
// 8192x5120x4096 onto it and lost 2-3 %. 160x128 / 128x160 (0.70): 1160 /
// 1170 TF/s on 8 full rounds (5120x8192x4096 / 8192x5120x4096,
// profiles/r2_tiles/); they fill a round where the square tiles leave CUs idle
// (5624x752x5880: 216 tiles of 160x128 vs 180 of 160x160, 677 vs 616 TF/s).
// 128x256 (round 3, hipBLASLt's MT128x256 on 4672x1472x6696,
// profiles/r2_tiles/hipblaslt_kernels_stats.csv): 2 % above 256x128 on full
// rounds (8192x8192x4096 / 4096x8192x4096 / 8192x4096x4096: 1300 / 1289 / 1282
// vs 1279 / 1258 / 1253 TF/s, profiles/r3_tiles/), so 0.80 against 0.78; it
// wastes fewer edge rows where M is ragged and N a multiple of 256.
// 192x256 / 256x192 (round 5, `pp`: gemm_bf16_pp3h.hpp, the 8-wave ping-pong
// with one 64-row half; hipBLASLt's MT256x192 / MT192x256 on ragged one-round C,
// profiles/r5_h192/): one round of them took 0.88-0.96 of the time of
// pingpong8cm's round of 256x256 tiles on 7 ragged shapes, for 0.75 of the work
// per CU - eff 0.78-0.85, priced at 0.82. One-round tiles, like 160x128.
// They serve all of C in one launch only: as the rest part after whole rounds
// of 256x256 tiles they tied the old plan at best and lost 22-24 % at
// 5120x5120x128 / 256; below K = 1024 they lost 17-21 % to pingpong8cm
// (7400x1224x616, 4392x2184x544), where loading the A / B panels for 31 % more
// tiles dominates (profiles/r5_h192/plan_ab_*.log).
// (the CU count the rounds are priced over is the launch's own: device_cus())
struct SmallTile {
  int variant, tm, tn;
  double eff;
  bool masked;     // wave-specialised kernel: any M, N % 4, K % 8 (edge tiles / K tail masked)
  bool one_round;  // only where its tiles fit in one round of 256 CUs
  bool splitk;     // a split-K candidate (the split model was fitted without 128x256)
  double ragged;   // measured / modelled time of one round on ragged C (stream-K pricing only)
  bool pp = false;  // 8-wave ping-pong tile (gemm_bf16_pp3h.hpp): N % 8, bf16 only
};
// 160x128 / 128x160 are one-round tiles: filling a round the square tiles
// leave part-idle they win 2-16 % (5624x752x5880, 4072x1240x3784, the rest
// parts of 4608^3 / 6144^3); over 2+ rounds, in place of the 256x256 kernel's
// one partial round, they lost 3-22 % (3000^3, 1344x6216x4848, 1616x6208x6504;
// profiles/r2_tiles/plan_ab_*.log) - there the big kernel's partial round runs
// faster per tile than the full-chip rate the model prices.
// `ragged`: one round of the tile on C with an edge tile row / column or K % 128
// != 0 took 1.1-1.5x the modelled time on MI355X (20 one-round shapes,
// profiles/r4_sks/split_sweep.log; exact shapes were within 0.93-1.02x). Only
// the stream-K choice uses it: the tile choice itself was tuned with the model.
constexpr SmallTile kSmallTiles[] = {{15, 128, 128, 0.60, true, false, true, 1.13},
                                     {16, 256, 128, 0.78, true, false, true, 1.0},
                                     {17, 160, 160, 0.72, true, false, true, 1.17},
                                     {23, 160, 128, 0.70, true, true, true, 1.37},
                                     {24, 128, 160, 0.70, true, true, true, 1.37},
                                     {26, 128, 256, 0.80, true, false, false, 1.30},
                                     {18, 256, 160, 0.61, false, false, false, 1.0},
                                     {27, 192, 256, 0.82, true, true, false, 1.0, true},
                                     {28, 256, 192, 0.82, true, true, false, 1.0, true}};
// host-only A/B knob (tools/pp_plan_ab.py): bit 0 = the 192-wide tiles on all
// of C, bit 1 = stream-K split mode on them (3 = the shipping plan)
static bool g_plan_pp = true, g_plan_pp_split = true;
NTM_API void ntm_set_plan_pp_tiles(int on) {
  g_plan_pp = (on & 1) != 0;
  g_plan_pp_split = (on & 2) != 0;
}
// The counted vmcnt phase P (0..3) of the 192-wide ping-pong build <ah, bh>
// waits for (Geo::vmc, gemm_bf16_pp3h.hpp; 128 / 128 is pingpong8c's 10): host
// only, for the CPU model of the DMA schedule (tests/test_pp3h_schedule_model.py).
NTM_API int ntm_pp3h_vmcnt(int ah, int bh, int phase) {
  using namespace ntm::gemm3h;
  if (phase < 0 || phase > 3) return -1;
  int v[4];
  auto fill = [&](auto geo) {
    using G = decltype(geo);
    v[0] = G::vmc(0), v[1] = G::vmc(1), v[2] = G::vmc(2), v[3] = G::vmc(3);
  };
  if (ah == 64 && bh == 128) fill(Geo<64, 128>{});
  else if (ah == 128 && bh == 64) fill(Geo<128, 64>{});
  else if (ah == 96 && bh == 128) fill(Geo<96, 128>{});
  else if (ah == 128 && bh == 128) fill(Geo<128, 128>{});
  else return -1;
  return v[phase];
}
constexpr int kPpMinK = 1024;
constexpr double kSplitPenalty = 0.25;  // a second launch, in 128x128-tile-round units

struct K1Plan {
  int top_rows;      // rows [0, top_rows) on top_variant; -1 = no plan tiles (M,N,K)
  int top_variant;   // 5 / 4 (the 256x256 kernel) or a kSmallTiles variant
  int rest_variant;  // rows [top_rows, M) on a kSmallTiles variant
  int splits = 1;    // > 1: all of C on top_variant (masked tile), split-K in that many slices
  bool sk = false;   // all of C on the stream-K kernel (top_variant kStreamKVariant)
  bool feasible() const { return top_rows >= 0; }
};

// Split-K time model (seconds), fitted on MI355X (tools/experiments/splitk_check.py, 14
// shapes x 3 tiles x up to 6 slice counts, profiles/r2_splitk/): a round of
// tm x tn tiles over kc costs 2 tm tn kc / (kPerCU eff); the fp32 partials cost
// kRedFixed + slices M N 4 / kRedBW (the partial stores in the tile epilogue +
// the reduction kernel's reads; an effective rate, not HBM's). Its picks are
// within 3.3 % of the fastest measured split on every fitted shape. A split plan
// must beat the unsplit one by kSplitKMargin.
// Round 5 (profiles/r5_margin/): the model leaves out per-launch fixed costs on
// both sides, so on small C the unsplit plan is about as optimistic as the
// split one, and the 1.1 margin kept C unsplit where a split with long slices
// ran 10-25 % faster. A split whose slices keep >= kLongSliceK of K needs only
// kSplitKMarginLong against the unsplit plan. Short slices keep 1.1 (at 1.03,
// three slices of 464 / 621 K lost 22-28 %), and so does any split against a
// stream-K plan (at 1.03, 256x128 / 2 replaced stream-K split mode on 14
// shapes and lost on 10, by up to 8 %).
constexpr double kPerCU = 1650e12 / 256.0;  // the 256x256 kernel's per-CU bf16 rate
constexpr double kRedFixed = 2e-6;
constexpr double kRedBW = 2e12;
constexpr double kSplitKMargin = 1.1;
constexpr double kSplitKMarginLong = 1.03;
constexpr int kLongSliceK = 1024;
// K1-fp8 (K in bf16-sized pairs of e4m3): the same rule from slices of >= 1152
// pairs (profiles/r5_margin/fp8_seed*: of 52 changed shapes on three seeds, the
// three that lost 15-20 % had slices of 1000-1036 pairs, 1024 / 1088 after
// rounding to the K tile; from 1152 on, 43 of 49 ran faster, median 1.13)
constexpr int kLongSliceKFp8 = 1152;
// host-only A/B knob (tools/margin_ab.py): the long-slice margin and threshold
// the plan uses (margin <= 0 / long_k < 0: the shipping values; margin 1.1 =
// round 4's plan); both are in the plan cache key
// fp8_long = 0 keeps K1-fp8's split-K at 1.1 everywhere (round 4's fp8 plan);
// < 0: the shipping fp8 rule
static double g_splitk_margin = 0.0;
static int g_splitk_min_k = -1;
static bool g_splitk_fp8_long = true;
// Split-K candidates with slices of >= kLongSliceK are priced against the
// ragged-scaled unsplit time that stream-K already uses (profiles/r5_margin/):
// 146 changed plans on seeds 12 / 13 - long slices 95 of 129 faster, geo-mean
// 1.045; short ones lost up to 37 % - then fresh seed 14: 46 of 55 faster,
// median 1.04, worst 0.875. bf16 only (not measured on K1-fp8). Host-only A/B
// knob (ntm_set_plan_splitk_ragged).
static bool g_splitk_ragged = true;
NTM_API void ntm_set_plan_splitk_ragged(int on) { g_splitk_ragged = on != 0; }
NTM_API void ntm_set_plan_splitk(double margin, int long_k, int fp8_long) {
  g_splitk_margin = margin > 0.0 ? margin : 0.0;
  g_splitk_min_k = long_k >= 0 ? long_k : -1;
  g_splitk_fp8_long = fp8_long != 0;
}
inline double splitk_long_margin() {
  return g_splitk_margin > 0.0 ? g_splitk_margin : kSplitKMarginLong;
}
inline int splitk_long_k() { return g_splitk_min_k >= 0 ? g_splitk_min_k : kLongSliceK; }
constexpr int kMaxSplits = 16;

// Stream-K ("pingpong8s", gemm_bf16_sk.hpp; needs the caller's workspace, so
// only in the split-K plan). Time model, from its stamps (profiles/r4_sk/
// sk_stamps.log): the K loop runs 5 % slower per K-tile pair than the
// data-parallel kernel's (two K offsets per XCD instead of one), over
// ntiles / G tiles per CU, plus ~30 us per workgroup for the fix-ups, the
// extra C store and the imbalance between 2- and 3-segment workgroups. It is
// within +-5 % of the measured time on 29 of 30 shapes (profiles/r4_sk/
// plan_calibration.log). The unsplit plan's model leaves out per-tile fixed
// costs, so it is optimistic; stream-K is chosen whenever its predicted time is
// below the unsplit plan's (4 of 41 random shapes: measured +1 to +12 %).
// Split mode (at most half a round of tiles, S K slices each): ceil(Tp / S)
// pairs per CU plus the fix-up terms below, priced against the unsplit plan
// scaled by SmallTile::ragged (profiles/r4_sks: 6 of 15 sweep shapes, +9 to
// +39 % over the small tile).
constexpr int kStreamKVariant = 49;
// split mode on the 192-wide ping-pong tiles (gemm_bf16_skh.hpp): a tile of
// them costs kPpTileTime of a 256x256 tile over the same K (0.75 of the work at
// the 0.82 efficiency the plan prices them at); its partials are 0.75 the size
constexpr int kStreamKPp192x256 = 54, kStreamKPp256x192 = 55;
constexpr double kPpTileTime = 0.75 / 0.82;
// the last split-K plan's predicted unsplit / stream-K seconds (ntm_k1_plan_times)
static thread_local double g_plan_debug_unsplit_s = 0.0, g_plan_debug_sk_s = 0.0;
constexpr double kSkLoopFactor = 1.05;
constexpr double kSkFixed = 30e-6;
constexpr double kSkMargin = 1.0;
// split mode (at most half a round of tiles, gemm_bf16_sks_kernel): the K loop
// of ceil(Tp / S) pairs at the data-parallel rate, plus the fix-up. Every one of
// the P = tiles x S slices writes a 256 KiB partial (the write phase grows with
// P) and each combiner reads S of them (grows with S): fitted over 16 measured
// shapes, S = 2..8, P = 128..256, rms 4 us (profiles/r4_sks, r4_tiles).
constexpr double kSkSplitFixed = -18e-6;
constexpr double kSkSplitPerPartial = 0.15e-6;
constexpr double kSkSplitPerSlice = 3.4e-6;
constexpr double kSkSplitMinFixup = 8e-6;

// The plan: C split by rows into a top part and a rest part, each on one tile
// kernel in its own launch (either part may be empty). The top part runs the
// 256x256 kernel or a small tile, the rest a small tile; the smallest
// predicted time wins. Mixed small tiles fill whole rounds where one tile
// shape cannot: 3200^3 = 1920 rows of 160x160 (240 tiles) + 1280 rows of
// 128x128 (250 tiles), two full rounds instead of 1.56 rounds of 160x160
// (977 vs 924 TF/s, hipBLASLt 948: profiles/r2_ws/split_3200.log).
// Ties: fewer launches, then more rows on the 256x256 kernel, then (one
// launch) less of C covered by tiles (edge waste): in one round, 128x160 beat 160x128 (equal
// modelled cost) wherever it had fewer tiles, by 2-13 % (8008x536x2896: 252 vs
// 255 tiles, 34.8 vs 39.4 us; 4152x1096x16056, 1456x2696x10744), and tied
// where the counts were equal (profiles/r4_tiles).
// fp8 (K1-fp8's plan): K counted in bf16-sized pairs of e4m3 values (a K-tile
// costs the same cycles in both dtypes); only the tiles with an fp8 build - the
// 256x256 kernel and the wave-specialised ones - and no split-K.
inline K1Plan plan_k1_search(int M, int N, int K, bool splitk, bool fp8) {
  // the CUs the launches below run on (256 on MI355X in SPX mode; fewer in a
  // DPX / CPX partition): stream-K's decomposition must be the launch's own
  const double kCUs = (double)ntm::gemm6::device_cus();
  auto rounds = [&](double tiles) { return tiles <= 0 ? 0.0 : __builtin_ceil(tiles / kCUs); };
  const double inf = 1e300;
  // the 256x256 kernel on whole tiles: pingpong8c (K % 128). K % 128 != 0 goes
  // to the masked build's partial-K path (22), measured faster than pingpong8b
  // (8192x8192x8000: 1634 vs 1472 TF/s, profiles/r2_ws/ktail_pp2_vs_cm.log); the
  // pingpong8b clause below only matters if that build ever cannot serve a shape
  const bool big_masked_ok = N % 8 == 0 && K % 8 == 0;
  const bool big_ok = N % 256 == 0 && K >= 128 &&
                      (K % 128 == 0 || (K % 64 == 0 && !big_masked_ok));
  const int big_variant = K % 128 == 0 ? kDefaultVariant : 4;
  K1Plan best{-1, 15, 15};
  double best_cost = inf;
  int best_launches = 3, best_big_rows = -1;
  double best_cover = inf;
  if (M <= 0 || N <= 0 || K <= 0) return best;
  auto small_ok = [&](const SmallTile& st, int rows) {  // masked: any M, N % 4, K % 8
    if (fp8 && (!st.masked || st.pp)) return false;
    if (st.pp) return g_plan_pp && N % 8 == 0 && K % 8 == 0 && K >= kPpMinK;
    if (st.masked) return N % 4 == 0 && K % 8 == 0;
    return rows % st.tm == 0 && N % st.tn == 0 && K % 128 == 0 && K >= 128;
  };
  auto small_cost = [&](const SmallTile& st, int rows) {  // edge tiles cost a whole tile
    const double tiles = (double)((rows + st.tm - 1) / st.tm) * ((N + st.tn - 1) / st.tn);
    if (st.one_round && tiles > kCUs) return inf;
    return rounds(tiles) * (st.tm * st.tn / 16384.0) / st.eff;
  };
  // top candidates: index -1 = the 256x256 kernel, else kSmallTiles[t]
  const int nsmall = (int)(sizeof(kSmallTiles) / sizeof(kSmallTiles[0]));
  // the 256x256 kernel on ragged C: variant 22 (masked edge tiles, N % 8, K % 8)
  for (int t = -1; t < nsmall; ++t) {
    const int tm = t < 0 ? 256 : kSmallTiles[t].tm;
    if (t < 0 && !big_ok && !big_masked_ok) continue;
    if (t >= 0 && !small_ok(kSmallTiles[t], kSmallTiles[t].tm)) continue;
    const bool masked = t >= 0 ? kSmallTiles[t].masked : big_masked_ok;
    for (int m1 = tm; m1 < M + (masked ? tm : 1); m1 += tm) {
      if (m1 > M) m1 = M;  // masked kernel: the whole of C, last tile row partial
      const bool big_exact = t < 0 && big_ok && m1 % 256 == 0;
      if (t < 0 && !big_exact && !big_masked_ok) continue;
      const double top = t < 0 ? rounds((double)((m1 + 255) / 256) * ((N + 255) / 256)) * 4.0
                               : small_cost(kSmallTiles[t], m1);
      const int rest = M - m1;
      for (int r = 0; r < nsmall; ++r) {
        if (rest > 0 && (kSmallTiles[r].pp || !small_ok(kSmallTiles[r], rest))) continue;
        if (rest == 0 && r > 0) break;  // no rest part: one candidate is enough
        const double cost = top + (rest > 0 ? small_cost(kSmallTiles[r], rest) + kSplitPenalty : 0.0);
        if (cost >= inf) continue;  // a one-round tile over more than one round
        // one-round tiles: all of C, or the rest after the 256x256 kernel's rounds
        if (rest > 0 && t >= 0 && (kSmallTiles[t].one_round || kSmallTiles[r].one_round))
          continue;
        const int launches = rest > 0 ? 2 : 1;
        const int big_rows = t < 0 ? m1 : 0;
        auto cover = [&](int tmc, int tnc, int rows) {  // elements of C the tiles span
          return rows <= 0 ? 0.0 : (double)((rows + tmc - 1) / tmc) * ((N + tnc - 1) / tnc) * tmc * tnc;
        };
        const double cov = (t < 0 ? cover(256, 256, m1) : cover(tm, kSmallTiles[t].tn, m1)) +
                           (rest > 0 ? cover(kSmallTiles[r].tm, kSmallTiles[r].tn, rest) : 0.0);
        const bool better = cost < best_cost - 1e-9 ||
                            (cost <= best_cost + 1e-9 &&
                             (launches < best_launches ||
                              (launches == best_launches &&
                               (big_rows > best_big_rows ||
                                (big_rows == best_big_rows && launches == 1 && cov < best_cover)))));
        if (better) {
          best_cost = cost;
          best_launches = launches;
          best_big_rows = big_rows;
          best_cover = cov;
          best = K1Plan{m1, t < 0 ? (big_exact ? big_variant : 22) : kSmallTiles[t].variant,
                        rest > 0 ? kSmallTiles[r].variant : (t < 0 ? 15 : kSmallTiles[t].variant)};
        }
      }
    }
  }
  // whole 256x256 tiles over more than one round: the persistent build
  // (K1-fp8: from one round on, K in bf16-sized pairs)
  if (!fp8 && best.feasible() && best.top_variant == kDefaultVariant && K >= 256 &&
      (double)(best.top_rows / 256) * (N / 256) > kCUs)
    best.top_variant = kPersistentVariant;
  if (fp8 && kFp8Persistent && best.feasible() && best.top_variant == kDefaultVariant &&
      ntm::gemm6::shape_ok6(best.top_rows, N, K))
    best.top_variant = kPersistentVariant;
  if (!splitk || !best.feasible()) return best;
  // Split-K: C too small to fill 256 CUs with a long K (e.g. 280x6352x7568: 80
  // tiles of 160x160 -> 3 slices of 240 tiles, 631 vs 321 TF/s unsplit).
  const double unit_s = 2.0 * 16384.0 * K / kPerCU;  // cost units -> seconds
  const double unsplit = best_cost * unit_s;
  double best_t = inf;        // the fastest split-K candidate so far
  double sk_bar = inf;        // a split-K plan must also beat a chosen stream-K plan
  K1Plan split = best;
  // Stream-K: a partial last round of 256x256 tiles spread over every CU, or
  // split mode (at most half a round of tiles) on the 256x256 or the 192-wide
  // tiles; the fastest predicted candidate is priced against the unsplit plan
  ntm::gemmsk::SkArgs sk;
  g_plan_debug_unsplit_s = unsplit;
  g_plan_debug_sk_s = 0.0;
  double t_sk = 0.0;
  int sk_variant = 0;
  auto split_mode_s = [&](const ntm::gemmsk::SkArgs& a, double tile_s, double partial_scale) {
    // one slice of ceil(Tp / S) pairs per CU, one round, plus the fix-up
    const double pairs = (double)((a.Tp + a.S - 1) / a.S);
    const double fixup = kSkSplitFixed + kSkSplitPerPartial * partial_scale * a.ntiles * a.S +
                         kSkSplitPerSlice * a.S;
    return pairs / a.Tp * tile_s + (fixup > kSkSplitMinFixup ? fixup : kSkSplitMinFixup);
  };
  if (!fp8 && ntm::gemmsk::shape_ok_sk(M, N, K)) {
    if (ntm::gemmsk::sk_decompose(M, N, K, (int)kCUs, sk)) {
      const double tile_s = 4.0 * unit_s * (2.0 * sk.Tp * ntm::gemm::BK / K);  // one 256x256 tile, K in pairs
      t_sk = sk.S >= 2 ? split_mode_s(sk, tile_s, 1.0)
                       : kSkLoopFactor * ((double)sk.ntiles / kCUs) * tile_s + kSkFixed;
      sk_variant = kStreamKVariant;
    }
    if (g_plan_pp_split && K >= kPpMinK) {
      for (int gi = 0; gi < 2; ++gi) {
        ntm::gemmsk::SkArgs sh;
        const bool ok = gi == 0 ? ntm::gemmskh::sk_decompose_h<192, 256>(M, N, K, (int)kCUs, sh)
                                : ntm::gemmskh::sk_decompose_h<256, 192>(M, N, K, (int)kCUs, sh);
        // S = 2 (the head / tail protocol) only: at S >= 3 it replaced a small tile
        // on 4 random shapes and lost on 3 (0.88-0.98, profiles/r5_skh/pp_ab_random200.log)
        if (!ok || sh.S != 2) continue;
        const double tile_s = kPpTileTime * 4.0 * unit_s * (2.0 * sh.Tp * ntm::gemm::BK / K);
        const double t = split_mode_s(sh, tile_s, 0.75);
        if (sk_variant == 0 || t < t_sk) {
          t_sk = t;
          sk_variant = gi == 0 ? kStreamKPp192x256 : kStreamKPp256x192;
        }
      }
    }
  }
  // a single launch of one small tile in one round on ragged C runs slower
  // than the model (SmallTile::ragged): stream-K is priced against the
  // measured-ish time (and split-K too, with the A/B knob below)
  double unsplit_ragged = unsplit;
  if (best.top_rows == M && best.top_variant == best.rest_variant)
    for (const SmallTile& st : kSmallTiles)
      if (st.variant == best.top_variant &&
          (double)((M + st.tm - 1) / st.tm) * ((N + st.tn - 1) / st.tn) <= kCUs &&
          (M % st.tm != 0 || N % st.tn != 0 || K % 128 != 0))
        // rows of A / B at least 64-byte aligned (K % 32 == 0): a third of it
        // (4704, 6240, 10720: 1.00-1.16 where 16 / 32-byte rows gave 1.1-1.5)
        // and 16-byte rows (K % 16 == 8) at least 1.25 (128x128 1.26 / 1.27,
        // 160x160 1.11 / 1.35 measured)
        unsplit_ragged *= K % 32 == 0   ? 1.0 + (st.ragged - 1.0) * 0.4
                          : K % 16 == 8 ? (st.ragged > 1.0 && st.ragged < 1.25 ? 1.25 : st.ragged)
                                        : st.ragged;
  if (sk_variant != 0) {
    g_plan_debug_sk_s = t_sk;
    const double unsplit_vs_sk = unsplit_ragged;
    g_plan_debug_unsplit_s = unsplit_vs_sk;
    if (t_sk * kSkMargin < unsplit_vs_sk) {
      split = K1Plan{M, sk_variant, sk_variant, 1};
      split.sk = true;
      sk_bar = t_sk * kSkMargin / kSplitKMargin;
    }
  }
  for (const SmallTile& st : kSmallTiles) {
    if (!st.masked || !st.splitk || !small_ok(st, M)) continue;
    const double tiles = (double)((M + st.tm - 1) / st.tm) * ((N + st.tn - 1) / st.tn);
    for (int sp = 2; sp <= kMaxSplits; ++sp) {
      const int slices = ntm::gemmt::splitk_slices(K, sp);
      if (slices != sp) continue;  // the same slicing as a smaller sp
      if (st.one_round && tiles * slices > kCUs) break;
      const double kc = ntm::gemmt::splitk_kc(K, sp);
      const double t = rounds(tiles * slices) * 2.0 * st.tm * st.tn * kc / (kPerCU * st.eff) +
                       kRedFixed + (double)slices * M * N * 4.0 / kRedBW;
      const int long_k = fp8 ? (g_splitk_min_k >= 0 ? g_splitk_min_k : kLongSliceKFp8)
                             : splitk_long_k();
      const double margin = (!fp8 || g_splitk_fp8_long) && kc >= long_k
                                ? splitk_long_margin() : kSplitKMargin;
      const double vs = g_splitk_ragged && !fp8 && kc >= splitk_long_k() ? unsplit_ragged : unsplit;
      if (t < best_t && t * margin < vs && t < sk_bar) {
        best_t = t;
        split = K1Plan{M, st.variant, st.variant, slices};
      }
    }
  }
  return split;
}

// The plan is an exhaustive search over tiles and row splits: 3-25 us of host
// time per shape, paid on every default-dispatch call until round 5 (twice in
// ntm_gemm_bf16_ex). For C of a few microseconds that made the launch
// host-bound (6712x280x368: 18.3 us per call against 8.0 for its own tile,
// profiles/r5_h192/small_shapes_sweep.log). Plans are memoised per host thread
// in a small direct-mapped table keyed by everything the search reads.
struct PlanKey {
  int M, N, K, cus;
  bool splitk, fp8;
  int pp;
  double margin;
  int min_k;
  bool fp8_long;
  bool operator==(const PlanKey& o) const {
    return M == o.M && N == o.N && K == o.K && cus == o.cus && splitk == o.splitk &&
           fp8 == o.fp8 && pp == o.pp && margin == o.margin && min_k == o.min_k &&
           fp8_long == o.fp8_long;
  }
};
struct PlanEntry {
  PlanKey key;
  K1Plan plan;
  double unsplit_s, sk_s;  // the search's debug outputs (ntm_k1_plan_times)
  bool valid;
};
constexpr int kPlanCacheSlots = 256;

inline K1Plan plan_k1(int M, int N, int K, bool splitk = false, bool fp8 = false) {
  static thread_local PlanEntry cache[kPlanCacheSlots] = {};
  const PlanKey key{M, N, K, ntm::gemm6::device_cus(), splitk, fp8,
                    (g_plan_pp ? 1 : 0) | (g_plan_pp_split ? 2 : 0) | (g_splitk_ragged ? 4 : 0),
                    g_splitk_margin,
                    g_splitk_min_k, g_splitk_fp8_long};
  const unsigned h = ((unsigned)M * 2654435761u) ^ ((unsigned)N * 40503u) ^ ((unsigned)K * 97u) ^
                     ((unsigned)key.cus << 3) ^ (splitk ? 0x55u : 0u) ^ (fp8 ? 0xAAu : 0u) ^
                     ((unsigned)key.pp << 8);
  PlanEntry& e = cache[(h ^ (h >> 8) ^ (h >> 16)) % kPlanCacheSlots];
  if (e.valid && e.key == key) {
    g_plan_debug_unsplit_s = e.unsplit_s;
    g_plan_debug_sk_s = e.sk_s;
    return e.plan;
  }
  const K1Plan p = plan_k1_search(M, N, K, splitk, fp8);
  e = PlanEntry{key, p, g_plan_debug_unsplit_s, g_plan_debug_sk_s, true};
  return p;
}

// The split-K plan's predicted seconds for (M, N, K): the best unsplit plan and
// stream-K (0 when it does not serve the shape). Host only; tools.
NTM_API int ntm_k1_plan_times(int M, int N, int K, double* unsplit_s, double* sk_s) {
  if (!unsplit_s || !sk_s || !plan_k1(M, N, K, true).feasible()) return (int)hipErrorInvalidValue;
  *unsplit_s = g_plan_debug_unsplit_s;
  *sk_s = g_plan_debug_sk_s;
  return 0;
}

// The default dispatch's plan for (M, N, K) (host only; tests and tools).
NTM_API int ntm_k1_plan(int M, int N, int K, int* top_rows, int* top_variant, int* rest_variant) {
  if (M <= 0 || N <= 0 || K <= 0 || !top_rows || !top_variant || !rest_variant)
    return (int)hipErrorInvalidValue;
  const K1Plan pl = plan_k1(M, N, K);
  if (!pl.feasible()) return (int)hipErrorInvalidValue;
  *top_rows = pl.top_rows;
  *top_variant = pl.top_variant;
  *rest_variant = pl.rest_variant;
  return 0;
}

// The same with split-K allowed (a workspace of ntm_splitk_ws_bytes(M, N, K,
// *splits) bytes when *splits > 1): the plan ntm_gemm_bf16_ex runs.
NTM_API int ntm_k1_plan_splitk(int M, int N, int K, int* top_rows, int* top_variant,
                               int* rest_variant, int* splits) {
  if (M <= 0 || N <= 0 || K <= 0 || !top_rows || !top_variant || !rest_variant || !splits)
    return (int)hipErrorInvalidValue;
  const K1Plan pl = plan_k1(M, N, K, true);
  if (!pl.feasible()) return (int)hipErrorInvalidValue;
  *top_rows = pl.top_rows;
  *top_variant = pl.top_variant;
  *rest_variant = pl.rest_variant;
  *splits = pl.splits;
  return 0;
}

NTM_API int ntm_gemm_bf16_variant(int variant, const void* A, const void* B,
                                  void* C, int M, int N, int K, int lda,
                                  int ldb, int ldc, void* stream) {
  if (variant == 0) {
    const K1Plan pl = plan_k1(M, N, K);
    if (!pl.feasible()) return (int)hipErrorInvalidValue;  // nothing launched
    if (pl.top_rows < M) {
      const int rc = ntm_gemm_bf16_variant(pl.top_variant, A, B, C, pl.top_rows, N, K, lda, ldb,
                                           ldc, stream);
      if (rc != 0) return rc;
      return ntm_gemm_bf16_variant(pl.rest_variant, (const __bf16*)A + (size_t)pl.top_rows * lda,
                                   B, (__bf16*)C + (size_t)pl.top_rows * ldc, M - pl.top_rows, N,
                                   K, lda, ldb, ldc, stream);
    }
    variant = pl.top_variant;
  }
  ntm::gemm::GemmArgs a;
  a.A = (const __bf16*)A;
  a.B = (const __bf16*)B;
  a.C = (__bf16*)C;
  a.M = M;
  a.N = N;
  a.K = K;
  a.lda = lda;
  a.ldb = ldb;
  a.ldc = ldc;
  switch (variant) {
    case 4: return (int)ntm::gemm2::launch_gemm_bf16_pp2(a, S(stream));
    case 5: return (int)ntm::gemm3::launch_gemm_bf16_pp3(a, S(stream));
    // persistent pingpong8c with overlapped C stores (needs lda / ldb / ldc % 8,
    // K >= 256; otherwise the same tiles on pingpong8c)
    case 25:
      if (!ntm::gemm6::shape_ok6(M, N, K) || (lda % 8) || (ldb % 8) || (ldc % 8))
        return (int)ntm::gemm3::launch_gemm_bf16_pp3(a, S(stream));
      return (int)ntm::gemm6::launch_gemm_bf16_pp6<1, 0, kPp6Spread>(a, S(stream));
    // gemm_bf16_t128.hpp: 128x128 / 256x128 / 160x160 tiles on the wave-specialised
    // kernel (4 DMA-producer + 4 MFMA-consumer waves), 256x160 on the 4-wave one
    case 15: return (int)ntm::gemmt::launch_gemm_bf16_tile_ws<4>(a, S(stream));
    case 16: return (int)ntm::gemmt::launch_gemm_bf16_tile_ws<8>(a, S(stream));
    case 17: return (int)ntm::gemmt::launch_gemm_bf16_tile_ws<5, 5>(a, S(stream));
    case 23: return (int)ntm::gemmt::launch_gemm_bf16_tile_ws<5, 4>(a, S(stream));  // 160x128
    case 24: return (int)ntm::gemmt::launch_gemm_bf16_tile_ws<4, 5>(a, S(stream));  // 128x160
    case 26: return (int)ntm::gemmt::launch_gemm_bf16_tile_ws<4, 8>(a, S(stream));  // 128x256
    case 18: return (int)ntm::gemmt::launch_gemm_bf16_tile<8, 5>(a, S(stream));
    // 256x256 on ragged C: clamped loads, masked LDS-staged stores
    case 22: return (int)ntm::gemm3::launch_gemm_bf16_pp3_masked(a, S(stream));
    // 192x256 / 256x192 on the same ping-pong (gemm_bf16_pp3h.hpp): ragged C, one round
    case 27: return (int)ntm::gemm3h::launch_gemm_bf16_pp3h<64, 128>(a, S(stream));
    case 28: return (int)ntm::gemm3h::launch_gemm_bf16_pp3h<128, 64>(a, S(stream));
    // dma4k_d3 (gemm_w4k.hpp): 4 waves x 128x128 per wave on 256x256 tiles, a DMA
    // piece every 3 slots. Not on the plan: under the power limit it trades places
    // with pingpong8o box by box (-3 % .. +1.8 %, profiles/r6_w4kh), so bench.py
    // measures both on the box it runs on and times the faster (select_k1).
    case 39: return (int)ntm::w4k::launch_gemm_bf16_w4k<3>(a, S(stream));
    default: return (int)hipErrorInvalidValue;  // experimental variants: libntm_experimental.so
  }
}

// Split-K on a wave-specialised tile (15-17, 23, 24, 26): `splits` K-slices, fp32 partials
// in the caller's workspace ws (ntm_splitk_ws_bytes; stream-ordered, reused once
// this call's reduction has run), then one reduction kernel writes C.
NTM_API size_t ntm_splitk_ws_bytes(int M, int N, int K, int splits) {
  if (M <= 0 || N <= 0 || K <= 0 || splits < 1) return 0;
  return sizeof(float) * (size_t)ntm::gemmt::splitk_slices(K, splits) * M * N;
}

NTM_API int ntm_gemm_bf16_splitk(int variant, int splits, const void* A, const void* B, void* C,
                                 int M, int N, int K, int lda, int ldb, int ldc, void* ws,
                                 size_t ws_bytes, void* stream) {
  if (splits < 1 || !ws || ws_bytes < ntm_splitk_ws_bytes(M, N, K, splits))
    return (int)hipErrorInvalidValue;
  ntm::gemm::GemmArgs a;
  a.A = (const __bf16*)A;
  a.B = (const __bf16*)B;
  a.C = (__bf16*)C;
  a.M = M;
  a.N = N;
  a.K = K;
  a.lda = lda;
  a.ldb = ldb;
  a.ldc = ldc;
  float* w = (float*)ws;
  using namespace ntm::gemmt;
  switch (variant) {
    case 15: return (int)launch_gemm_bf16_tile_ws_splitk<4, 4>(a, splits, w, S(stream));
    case 16: return (int)launch_gemm_bf16_tile_ws_splitk<8, 4>(a, splits, w, S(stream));
    case 17: return (int)launch_gemm_bf16_tile_ws_splitk<5, 5>(a, splits, w, S(stream));
    case 23: return (int)launch_gemm_bf16_tile_ws_splitk<5, 4>(a, splits, w, S(stream));
    case 24: return (int)launch_gemm_bf16_tile_ws_splitk<4, 5>(a, splits, w, S(stream));
    case 26: return (int)launch_gemm_bf16_tile_ws_splitk<4, 8>(a, splits, w, S(stream));
    default: return (int)hipErrorInvalidValue;
  }
}

// Stream-K on the 256x256 kernel ("pingpong8s", gemm_bf16_sk.hpp): the last two
// rounds of tiles dealt out as K-tile pairs over every CU, fp32 partials of the
// split tiles in ws. ntm_sk_ws_bytes = 0: stream-K does not serve (M, N, K) on
// this device (the tile count is a multiple of the CUs, or at most one round).
// Index (in 4-byte words) of the stream-K workspace's XCD-placement error word
// (gemm_bf16_sk.hpp kErrWord): nonzero after a launch in which some part of a
// split tile ran on a different XCD than the part that combined it.
NTM_API int ntm_sk_error_word_index() { return ntm::gemmsk::kErrWord; }
// Fault injection for that check (tests, the Job's self-check): nonzero makes the
// head / slice 0 of every split tile claim XCC_ID ^ v, so every stream-K launch
// after this call sets the error word. Process-wide; 0 = off.
NTM_API void ntm_set_sk_fault_inject(int v) { ntm::gemmsk::sk_fault_inject() = (unsigned)v; }

// The CU count the plan and the persistent / stream-K launches use, and a test
// override of it (0 = the device's own; host only: a CPU test of the plan on
// partition sizes other than 256 - never set it around real launches).
NTM_API int ntm_plan_cus() { return ntm::gemm6::device_cus(); }
NTM_API void ntm_set_cus_override(int cus) { ntm::gemm6::cu_override() = cus > 0 ? cus : 0; }

NTM_API size_t ntm_sk_ws_bytes(int M, int N, int K) {
  ntm::gemmsk::SkArgs s;
  if (!ntm::gemmsk::shape_ok_sk(M, N, K) ||
      !ntm::gemmsk::sk_decompose(M, N, K, ntm::gemm6::pp6_grid(1 << 30), s))
    return 0;
  return ntm::gemmsk::sk_ws_bytes(s.G);
}

NTM_API int ntm_gemm_bf16_sk(const void* A, const void* B, void* C, int M, int N, int K, int lda,
                             int ldb, int ldc, void* ws, size_t ws_bytes, void* stream) {
  ntm::gemm::GemmArgs a;
  a.A = (const __bf16*)A;
  a.B = (const __bf16*)B;
  a.C = (__bf16*)C;
  a.M = M;
  a.N = N;
  a.K = K;
  a.lda = lda;
  a.ldb = ldb;
  a.ldc = ldc;
  return (int)ntm::gemmsk::launch_gemm_bf16_sk(a, ntm::gemm6::pp6_grid(1 << 30), ws, ws_bytes,
                                               S(stream));
}

// Split mode on the 192-wide tiles (variant 54: 192x256, 55: 256x192;
// gemm_bf16_skh.hpp) with a stream-K workspace of ntm_skh_ws_bytes bytes (0:
// split mode on that tile does not serve (M, N, K) on this device).
NTM_API size_t ntm_skh_ws_bytes(int variant, int M, int N, int K) {
  ntm::gemmsk::SkArgs s;
  const int cus = ntm::gemm6::pp6_grid(1 << 30);
  if (!ntm::gemmsk::shape_ok_sk(M, N, K)) return 0;
  const bool ok = variant == kStreamKPp192x256   ? ntm::gemmskh::sk_decompose_h<192, 256>(M, N, K, cus, s)
                  : variant == kStreamKPp256x192 ? ntm::gemmskh::sk_decompose_h<256, 192>(M, N, K, cus, s)
                                                 : false;
  return ok ? ntm::gemmsk::sk_ws_bytes(s.G) : 0;
}

NTM_API int ntm_gemm_bf16_skh(int variant, const void* A, const void* B, void* C, int M, int N,
                              int K, int lda, int ldb, int ldc, void* ws, size_t ws_bytes,
                              void* stream) {
  ntm::gemm::GemmArgs a;
  a.A = (const __bf16*)A;
  a.B = (const __bf16*)B;
  a.C = (__bf16*)C;
  a.M = M;
  a.N = N;
  a.K = K;
  a.lda = lda;
  a.ldb = ldb;
  a.ldc = ldc;
  const int cus = ntm::gemm6::pp6_grid(1 << 30);
  if (variant == kStreamKPp192x256)
    return (int)ntm::gemmskh::launch_gemm_bf16_skh<64, 128>(a, cus, ws, ws_bytes, S(stream));
  if (variant == kStreamKPp256x192)
    return (int)ntm::gemmskh::launch_gemm_bf16_skh<128, 64>(a, cus, ws, ws_bytes, S(stream));
  return (int)hipErrorInvalidValue;
}

// ntm_gemm_bf16_skh with this launch's own fault-injection value (the Job runs
// one thread per GPU and corrupts only the last GPU's launch; -1 = the
// process-wide ntm_set_sk_fault_inject value).
NTM_API int ntm_gemm_bf16_skh_ex(int variant, const void* A, const void* B, void* C, int M, int N,
                                 int K, int lda, int ldb, int ldc, void* ws, size_t ws_bytes,
                                 int fault, void* stream) {
  ntm::gemm::GemmArgs a;
  a.A = (const __bf16*)A;
  a.B = (const __bf16*)B;
  a.C = (__bf16*)C;
  a.M = M;
  a.N = N;
  a.K = K;
  a.lda = lda;
  a.ldb = ldb;
  a.ldc = ldc;
  const int cus = ntm::gemm6::pp6_grid(1 << 30);
  if (variant == kStreamKPp192x256)
    return (int)ntm::gemmskh::launch_gemm_bf16_skh<64, 128>(a, cus, ws, ws_bytes, S(stream), fault);
  if (variant == kStreamKPp256x192)
    return (int)ntm::gemmskh::launch_gemm_bf16_skh<128, 64>(a, cus, ws, ws_bytes, S(stream), fault);
  return (int)hipErrorInvalidValue;
}

// The default dispatch with split-K allowed: ws (ws_bytes) is the caller's
// workspace; when the split-K plan needs more than ws_bytes (or ws is null) the
// unsplit plan runs instead.
NTM_API int ntm_gemm_bf16_ex(const void* A, const void* B, void* C, int M, int N, int K, int lda,
                             int ldb, int ldc, void* ws, size_t ws_bytes, void* stream) {
  if (ws) {
    const K1Plan pl = plan_k1(M, N, K, true);
    if (pl.feasible() && pl.splits > 1 && ws_bytes >= ntm_splitk_ws_bytes(M, N, K, pl.splits))
      return ntm_gemm_bf16_splitk(pl.top_variant, pl.splits, A, B, C, M, N, K, lda, ldb, ldc, ws,
                                  ws_bytes, stream);
    // stream-K: this entry takes any caller workspace, so it zeroes the counter
    // block first (a caller that keeps a zeroed workspace per stream calls
    // ntm_gemm_bf16_sk directly and saves that dispatch)
    if (pl.feasible() && pl.sk && pl.top_variant == kStreamKVariant &&
        ws_bytes >= ntm_sk_ws_bytes(M, N, K) &&
        hipMemsetAsync(ws, 0, ntm::gemmsk::kCounterBytes, S(stream)) == hipSuccess &&
        ntm_gemm_bf16_sk(A, B, C, M, N, K, lda, ldb, ldc, ws, ws_bytes, stream) == 0)
      return 0;
    if (pl.feasible() && pl.sk && pl.top_variant != kStreamKVariant &&
        ws_bytes >= ntm_skh_ws_bytes(pl.top_variant, M, N, K) &&
        ntm_skh_ws_bytes(pl.top_variant, M, N, K) > 0 &&
        hipMemsetAsync(ws, 0, ntm::gemmsk::kCounterBytes, S(stream)) == hipSuccess &&
        ntm_gemm_bf16_skh(pl.top_variant, A, B, C, M, N, K, lda, ldb, ldc, ws, ws_bytes, stream) == 0)
      return 0;
  }
  return ntm_gemm_bf16_variant(0, A, B, C, M, N, K, lda, ldb, ldc, stream);
}

// K1-fp8: C (bf16) = A (e4m3) * B (e4m3)^T, fp32 accumulation. Variant 5 / 22:
// the 256x256 kernel (gemm_fp8.hpp; exact, masked and partial-K builds picked by
// shape); 15 / 16 / 17 / 23 / 24 / 26: the wave-specialised tiles with the fp8
// consumer (gemm_bf16_t128.hpp); 0: the plan (plan_k1 in fp8 mode: tile shape
// and row split priced exactly as for bf16).
NTM_API int ntm_gemm_fp8_variant(int variant, const void* A, const void* B, void* C, int M, int N,
                                 int K, int lda, int ldb, int ldc, void* stream) {
  if (!ntm::fp8::shape_ok(M, N, K)) return (int)hipErrorInvalidValue;
  if (variant == 0) {
    const K1Plan pl = plan_k1(M, N, K / 2, false, true);
    if (!pl.feasible()) return (int)hipErrorInvalidValue;  // nothing launched
    if (pl.top_rows < M) {
      const int rc = ntm_gemm_fp8_variant(pl.top_variant, A, B, C, pl.top_rows, N, K, lda, ldb,
                                          ldc, stream);
      if (rc != 0) return rc;
      return ntm_gemm_fp8_variant(pl.rest_variant, (const char*)A + (size_t)pl.top_rows * lda, B,
                                  (__bf16*)C + (size_t)pl.top_rows * ldc, M - pl.top_rows, N, K,
                                  lda, ldb, ldc, stream);
    }
    variant = pl.top_variant;
  }
  __bf16* c = (__bf16*)C;
  using namespace ntm::gemmt;
  switch (variant) {
    case 5: case 22: return (int)ntm::fp8::launch_gemm_fp8(A, B, c, M, N, K, lda, ldb, ldc, S(stream));
    // the persistent overlap build (whole 256x256 tiles, K % 256, K >= 512;
    // otherwise the same tiles on pingpong8c)
    case 25:
      if (ntm::gemm6::fp8_pp6_ok(M, N, K, lda, ldb, ldc))
        return (int)ntm::gemm6::launch_gemm_fp8_pp6<kPp6Spread>(A, B, c, M, N, K, lda, ldb, ldc,
                                                               S(stream));
      return (int)ntm::fp8::launch_gemm_fp8(A, B, c, M, N, K, lda, ldb, ldc, S(stream));
    case 15: return (int)launch_gemm_fp8_tile_ws<4, 4>(A, B, c, M, N, K, lda, ldb, ldc, S(stream));
    case 16: return (int)launch_gemm_fp8_tile_ws<8, 4>(A, B, c, M, N, K, lda, ldb, ldc, S(stream));
    case 17: return (int)launch_gemm_fp8_tile_ws<5, 5>(A, B, c, M, N, K, lda, ldb, ldc, S(stream));
    case 23: return (int)launch_gemm_fp8_tile_ws<5, 4>(A, B, c, M, N, K, lda, ldb, ldc, S(stream));
    case 24: return (int)launch_gemm_fp8_tile_ws<4, 5>(A, B, c, M, N, K, lda, ldb, ldc, S(stream));
    case 26: return (int)launch_gemm_fp8_tile_ws<4, 8>(A, B, c, M, N, K, lda, ldb, ldc, S(stream));
    default: return (int)hipErrorInvalidValue;
  }
}

NTM_API int ntm_k1_fp8_plan(int M, int N, int K, int* top_rows, int* top_variant,
                            int* rest_variant) {
  if (!ntm::fp8::shape_ok(M, N, K) || !top_rows || !top_variant || !rest_variant)
    return (int)hipErrorInvalidValue;
  const K1Plan pl = plan_k1(M, N, K / 2, false, true);
  if (!pl.feasible()) return (int)hipErrorInvalidValue;
  *top_rows = pl.top_rows;
  *top_variant = pl.top_variant;
  *rest_variant = pl.rest_variant;
  return 0;
}

NTM_API int ntm_gemm_fp8(const void* A, const void* B, void* C, int M, int N, int K, int lda,
                         int ldb, int ldc, void* stream) {
  return ntm_gemm_fp8_variant(0, A, B, C, M, N, K, lda, ldb, ldc, stream);
}

// K1-fp8 split-K on a wave-specialised tile (15-17, 23, 24, 26): `splits` slices of
// the K-tile range, fp32 partials in ws (ntm_fp8_splitk_ws_bytes), one reduction.
NTM_API size_t ntm_fp8_splitk_ws_bytes(int M, int N, int K, int splits) {
  return ntm_splitk_ws_bytes(M, N, K / 2, splits);
}

NTM_API int ntm_gemm_fp8_splitk(int variant, int splits, const void* A, const void* B, void* C,
                                int M, int N, int K, int lda, int ldb, int ldc, void* ws,
                                size_t ws_bytes, void* stream) {
  if (!ntm::fp8::shape_ok(M, N, K) || splits < 1 || !ws ||
      ws_bytes < ntm_fp8_splitk_ws_bytes(M, N, K, splits))
    return (int)hipErrorInvalidValue;
  __bf16* c = (__bf16*)C;
  float* w = (float*)ws;
  using namespace ntm::gemmt;
  switch (variant) {
    case 15: return (int)launch_gemm_fp8_tile_ws_splitk<4, 4>(A, B, c, M, N, K, lda, ldb, ldc, splits, w, S(stream));
    case 16: return (int)launch_gemm_fp8_tile_ws_splitk<8, 4>(A, B, c, M, N, K, lda, ldb, ldc, splits, w, S(stream));
    case 17: return (int)launch_gemm_fp8_tile_ws_splitk<5, 5>(A, B, c, M, N, K, lda, ldb, ldc, splits, w, S(stream));
    case 23: return (int)launch_gemm_fp8_tile_ws_splitk<5, 4>(A, B, c, M, N, K, lda, ldb, ldc, splits, w, S(stream));
    case 24: return (int)launch_gemm_fp8_tile_ws_splitk<4, 5>(A, B, c, M, N, K, lda, ldb, ldc, splits, w, S(stream));
    case 26: return (int)launch_gemm_fp8_tile_ws_splitk<4, 8>(A, B, c, M, N, K, lda, ldb, ldc, splits, w, S(stream));
    default: return (int)hipErrorInvalidValue;
  }
}

// K1-fp8's plan with split-K allowed (what ntm_gemm_fp8_ex runs when given a
// workspace of ntm_fp8_splitk_ws_bytes(M, N, K, *splits) bytes).
NTM_API int ntm_k1_fp8_plan_splitk(int M, int N, int K, int* top_rows, int* top_variant,
                                   int* rest_variant, int* splits) {
  if (!ntm::fp8::shape_ok(M, N, K) || !top_rows || !top_variant || !rest_variant || !splits)
    return (int)hipErrorInvalidValue;
  const K1Plan pl = plan_k1(M, N, K / 2, true, true);
  if (!pl.feasible()) return (int)hipErrorInvalidValue;
  *top_rows = pl.top_rows;
  *top_variant = pl.top_variant;
  *rest_variant = pl.rest_variant;
  *splits = pl.splits;
  return 0;
}

NTM_API int ntm_gemm_fp8_ex(const void* A, const void* B, void* C, int M, int N, int K, int lda,
                            int ldb, int ldc, void* ws, size_t ws_bytes, void* stream) {
  if (ws && ntm::fp8::shape_ok(M, N, K)) {
    const K1Plan pl = plan_k1(M, N, K / 2, true, true);
    if (pl.feasible() && pl.splits > 1 && ws_bytes >= ntm_fp8_splitk_ws_bytes(M, N, K, pl.splits))
      return ntm_gemm_fp8_splitk(pl.top_variant, pl.splits, A, B, C, M, N, K, lda, ldb, ldc, ws,
                                 ws_bytes, stream);
  }
  return ntm_gemm_fp8_variant(0, A, B, C, M, N, K, lda, ldb, ldc, stream);
}

NTM_API int ntm_gemm_fp8_shape_ok(int M, int N, int K) {
  return ntm::fp8::shape_ok(M, N, K) ? 1 : 0;
}

NTM_API int ntm_gemm_bf16(const void* A, const void* B, void* C, int M, int N,
                          int K, int lda, int ldb, int ldc, void* stream) {
  return ntm_gemm_bf16_variant(0, A, B, C, M, N, K, lda, ldb, ldc, stream);
}

// K1 with the fused ABFT row checksum (default 8-wave kernel): rowsum[m] (fp32, M
// entries) must be zeroed by the caller on `stream` before the call.
NTM_API int ntm_gemm_bf16_rowsum(const void* A, const void* B, void* C,
                                 float* rowsum, int M, int N, int K, int lda,
                                 int ldb, int ldc, void* stream) {
  if (!rowsum) return (int)hipErrorInvalidValue;
  ntm::gemm::GemmArgs a;
  a.A = (const __bf16*)A;
  a.B = (const __bf16*)B;
  a.C = (__bf16*)C;
  a.M = M;
  a.N = N;
  a.K = K;
  a.lda = lda;
  a.ldb = ldb;
  a.ldc = ldc;
  a.rowsum = rowsum;
  return ntm::gemm3::shape_ok3(M, N, K) ? (int)ntm::gemm3::launch_gemm_bf16_pp3(a, S(stream))
                                        : (int)ntm::gemm2::launch_gemm_bf16_pp2(a, S(stream));
}

// K1-fp8 with the fused ABFT row checksum: the 256x256 fp8 build with kRowSum
// (exact shapes: M, N, K % 256); rowsum zeroed by the caller on `stream`.
NTM_API int ntm_gemm_fp8_rowsum(const void* A, const void* B, void* C, float* rowsum, int M,
                                int N, int K, int lda, int ldb, int ldc, void* stream) {
  if (!rowsum || !ntm::fp8::shape_exact(M, N, K) || lda < K || ldb < K || ldc < N ||
      (lda % 16) || (ldb % 16) || (ldc % 8))
    return (int)hipErrorInvalidValue;
  ntm::gemm::GemmArgs a;
  a.A = (const __bf16*)A;  // byte image: two e4m3 per bf16 slot (gemm_fp8.hpp)
  a.B = (const __bf16*)B;
  a.C = (__bf16*)C;
  a.M = M;
  a.N = N;
  a.K = K / 2;
  a.lda = lda / 2;
  a.ldb = ldb / 2;
  a.ldc = ldc;
  a.rowsum = rowsum;
  using ntm::gemm3::gemm_bf16_pp3_kernel;
  using ntm::gemm3::kEpiDefault;
  hipLaunchKernelGGL((gemm_bf16_pp3_kernel<true, ntm::gemm::kGroupM, false, kEpiDefault, 0, 3>),
                     dim3((unsigned)((M / ntm::gemm::BM) * (N / ntm::gemm::BN))),
                     dim3(ntm::gemm::kThreads), 0, S(stream), a);
  return (int)hipGetLastError();
}

namespace {
template <typename T>
int abft_check_t(const void* A, const void* B, const void* C, const float* rowsum, int M, int N,
                 int K, int lda, int ldb, int ldc, double* scratch, void* result,
                 hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || !rowsum || !scratch || !result)
    return (int)hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(scratch, 0, sizeof(double) * (size_t)K, stream);
  if (e != hipSuccess) return (int)e;
  e = hipMemsetAsync(result, 0, sizeof(ntm::aux::AbftResult), stream);
  if (e != hipSuccess) return (int)e;
  // ~2048 column blocks x row chunks: enough parallelism for 256 CUs
  const int kb = (K + 255) / 256;
  int chunks = (2048 + kb - 1) / kb;
  if (chunks > N) chunks = N;
  const int rpc = (N + chunks - 1) / chunks;
  chunks = (N + rpc - 1) / rpc;
  hipLaunchKernelGGL(ntm::aux::abft_colsum_kernel<T>, dim3(kb, chunks), dim3(256), 0, stream,
                     (const T*)B, N, K, ldb, rpc, scratch);
  hipLaunchKernelGGL(ntm::aux::abft_row_check_kernel<T>, dim3(M), dim3(256), 0, stream,
                     (const T*)A, lda, (const __bf16*)C, ldc, rowsum, scratch, N, K,
                     (ntm::aux::AbftResult*)result);
  return (int)hipGetLastError();
}
}  // namespace

// ABFT check of K1-fp8's C = A B^T (e4m3 operands) against its fused rowsum.
NTM_API int ntm_abft_check_fp8(const void* A, const void* B, const void* C, const float* rowsum,
                               int M, int N, int K, int lda, int ldb, int ldc, double* scratch,
                               void* result, void* stream) {
  return abft_check_t<uint8_t>(A, B, C, rowsum, M, N, K, lda, ldb, ldc, scratch, result,
                               S(stream));
}

// ABFT check of C = A B^T against the fused rowsum. scratch: K doubles;
// result: ntm::aux::AbftResult (both zeroed here, stream-ordered).
NTM_API int ntm_abft_check(const void* A, const void* B, const void* C,
                           const float* rowsum, int M, int N, int K, int lda,
                           int ldb, int ldc, double* scratch, void* result,
                           void* stream) {
  return abft_check_t<__bf16>(A, B, C, rowsum, M, N, K, lda, ldb, ldc, scratch, result,
                              S(stream));
}

NTM_API int ntm_abft_result_bytes() {
  return (int)sizeof(ntm::aux::AbftResult);
}

NTM_API int ntm_fill_uniform_bf16(void* out, size_t n, unsigned long long seed,
                                  float scale, void* stream) {
  if (n == 0) return 0;
  const unsigned grid = stream_grid((n + 7) / 8, 256);
  hipLaunchKernelGGL(ntm::aux::fill_uniform_bf16_kernel, dim3(grid), dim3(256),
                     0, S(stream), (__bf16*)out, n, (uint64_t)seed, scale);
  return (int)hipGetLastError();
}

NTM_API int ntm_ref_gemm_f32(const void* A, const void* B, float* C, int M,
                             int N, int K, int lda, int ldb, int ldc,
                             void* stream) {
  if (M <= 0 || N <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  dim3 grid((N + ntm::aux::kRefTile - 1) / ntm::aux::kRefTile,
            (M + ntm::aux::kRefTile - 1) / ntm::aux::kRefTile);
  hipLaunchKernelGGL(ntm::aux::ref_gemm_f32_kernel<__bf16>, grid, dim3(256), 0,
                     S(stream), (const __bf16*)A, (const __bf16*)B, C, M, N, K,
                     lda, ldb, ldc);
  return (int)hipGetLastError();
}

// K3 for K1-fp8: e4m3 operands (uniform [-1, 1) rounded RNE) and the fp32
// FMA reference over their exact values.
NTM_API int ntm_fill_uniform_e4m3(void* out, size_t n, unsigned long long seed, float scale,
                                  void* stream) {
  if (n == 0) return 0;
  const unsigned grid = stream_grid((n + 15) / 16, 256);
  hipLaunchKernelGGL(ntm::aux::fill_uniform_e4m3_kernel, dim3(grid), dim3(256), 0, S(stream),
                     (uint8_t*)out, n, (uint64_t)seed, scale);
  return (int)hipGetLastError();
}

NTM_API int ntm_ref_gemm_f32_e4m3(const void* A, const void* B, float* C, int M, int N, int K,
                                  int lda, int ldb, int ldc, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  dim3 grid((N + ntm::aux::kRefTile - 1) / ntm::aux::kRefTile,
            (M + ntm::aux::kRefTile - 1) / ntm::aux::kRefTile);
  hipLaunchKernelGGL(ntm::aux::ref_gemm_f32_kernel<uint8_t>, grid, dim3(256), 0, S(stream),
                     (const uint8_t*)A, (const uint8_t*)B, C, M, N, K, lda, ldb, ldc);
  return (int)hipGetLastError();
}

// result: device pointer to a zeroed ntm::aux::VerifyResult (32 bytes)
NTM_API int ntm_verify_bf16(const void* C, const float* R, size_t n,
                            float atol, float rtol, void* result,
                            void* stream) {
  const unsigned grid = stream_grid(n, 256);
  hipLaunchKernelGGL(ntm::aux::verify_bf16_kernel, dim3(grid), dim3(256), 0,
                     S(stream), (const __bf16*)C, R, n, atol, rtol,
                     (ntm::aux::VerifyResult*)result);
  return (int)hipGetLastError();
}

// Clock probe (aux_kernels.hpp clock_probe_kernel): grid blocks of 4 waves,
// out = 2 u64 per wave (shader cycles, 100 MHz ticks), sink = 1 float.
NTM_API int ntm_clock_probe(int grid, int iters, void* out, float* sink, void* stream) {
  if (grid <= 0 || iters <= 0 || !out || !sink) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(ntm::aux::clock_probe_kernel, dim3(grid), dim3(256), 0, S(stream), iters,
                     7u, (unsigned long long*)out, sink);
  return (int)hipGetLastError();
}

// GEMM clock: the shipping pingpong8o build with a start / end
// s_memtime + s_memrealtime stamp per workgroup (gemm_bf16_pp6.hpp STAMP 1).
// Whole 256x256 tiles, more tiles than CUs; stamps = ntm_gemm_bf16_clock_words()
// u64 per workgroup (start / end shader clock and real time, XCC_ID, HW_ID;
// ntm_gemm_bf16_clock_grid workgroups). C is the real product.
NTM_API int ntm_gemm_bf16_clock_words() { return ntm::gemm6::kClockStampWords; }

NTM_API int ntm_gemm_bf16_clock_grid(int M, int N) {
  if (M <= 0 || N <= 0 || M % 256 || N % 256) return 0;
  return ntm::gemm6::pp6_grid((M / 256) * (N / 256));
}

NTM_API int ntm_gemm_bf16_clock(const void* A, const void* B, void* C, int M, int N, int K,
                                int lda, int ldb, int ldc, void* stamps, void* stream) {
  if (!stamps) return (int)hipErrorInvalidValue;
  ntm::gemm::GemmArgs a;
  a.A = (const __bf16*)A;
  a.B = (const __bf16*)B;
  a.C = (__bf16*)C;
  a.M = M;
  a.N = N;
  a.K = K;
  a.lda = lda;
  a.ldb = ldb;
  a.ldc = ldc;
  a.stamps = (unsigned long long*)stamps;
  return (int)ntm::gemm6::launch_gemm_bf16_pp6<1, 1, kPp6Spread>(a, S(stream));
}

NTM_API int ntm_verify_result_bytes() {
  return (int)sizeof(ntm::aux::VerifyResult);
}

// K2 entry points. unroll in {2,4,8,16} selects the block-tiled kernels
// (policy bit0 = nontemporal loads, bit1 = nontemporal stores, bit2 (copy
// only) = software-pipelined; grid 0 = one block per tile, no grid-stride
// loop: the hardware dispatcher keeps every CU's wave slots full);
// unroll 1 selects the first grid-stride kernel (2048 x 256, nt), kept as
// the sweep baseline. Defaults measured by tools/hbm_sweep.py on MI355X.
namespace {
template <int U>
int copy_u(const void* src, void* dst, size_t n4, int policy, unsigned grid,
           hipStream_t s) {
  using namespace ntm::aux;
  const auto* a = (const ntm::f32x4*)src;
  auto* b = (ntm::f32x4*)dst;
  switch (policy) {
    case 0: hipLaunchKernelGGL((stream_copy_tiled_kernel<U, 0, 0>), dim3(grid), dim3(256), 0, s, a, b, n4); break;
    case 1: hipLaunchKernelGGL((stream_copy_tiled_kernel<U, 1, 0>), dim3(grid), dim3(256), 0, s, a, b, n4); break;
    case 2: hipLaunchKernelGGL((stream_copy_tiled_kernel<U, 0, 1>), dim3(grid), dim3(256), 0, s, a, b, n4); break;
    case 3: hipLaunchKernelGGL((stream_copy_tiled_kernel<U, 1, 1>), dim3(grid), dim3(256), 0, s, a, b, n4); break;
    case 4: hipLaunchKernelGGL((stream_copy_pipe_kernel<U, 0, 0>), dim3(grid), dim3(256), 0, s, a, b, n4); break;
    case 5: hipLaunchKernelGGL((stream_copy_pipe_kernel<U, 1, 0>), dim3(grid), dim3(256), 0, s, a, b, n4); break;
    case 6: hipLaunchKernelGGL((stream_copy_pipe_kernel<U, 0, 1>), dim3(grid), dim3(256), 0, s, a, b, n4); break;
    case 7: hipLaunchKernelGGL((stream_copy_pipe_kernel<U, 1, 1>), dim3(grid), dim3(256), 0, s, a, b, n4); break;
    case 9: hipLaunchKernelGGL((stream_copy_chunk_kernel<U, 1, 0>), dim3(grid), dim3(256), 0, s, a, b, n4); break;
    case 11: hipLaunchKernelGGL((stream_copy_chunk_kernel<U, 1, 1>), dim3(grid), dim3(256), 0, s, a, b, n4); break;
    case 8: hipLaunchKernelGGL((stream_copy_chunk_kernel<U, 0, 0>), dim3(grid), dim3(256), 0, s, a, b, n4); break;
    case 10: hipLaunchKernelGGL((stream_copy_chunk_kernel<U, 0, 1>), dim3(grid), dim3(256), 0, s, a, b, n4); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}
template <int U>
int read_u(const void* src, size_t n4, float* sink, int policy, unsigned grid,
           hipStream_t s) {
  using namespace ntm::aux;
  const auto* a = (const ntm::f32x4*)src;
  if (policy & 1)
    hipLaunchKernelGGL((stream_read_tiled_kernel<U, 1>), dim3(grid), dim3(256), 0, s, a, n4, sink);
  else
    hipLaunchKernelGGL((stream_read_tiled_kernel<U, 0>), dim3(grid), dim3(256), 0, s, a, n4, sink);
  return (int)hipGetLastError();
}
unsigned tiled_grid(size_t n4, int unroll, int grid) {
  if (grid > 0) return (unsigned)grid;
  const size_t tiles = n4 / (256 * (size_t)unroll);
  return (unsigned)(tiles < 1 ? 1 : (tiles > 0x7fffffffu ? 0x7fffffffu : tiles));
}
}  // namespace

NTM_API int ntm_stream_copy_ex(const void* src, void* dst, size_t bytes,
                               int unroll, int policy, int grid, void* stream) {
  if (bytes % 16 || grid < 0) return (int)hipErrorInvalidValue;
  const size_t n4 = bytes / 16;
  if (unroll == 1) {
    hipLaunchKernelGGL(ntm::aux::stream_copy_kernel, dim3(2048), dim3(256), 0,
                       S(stream), (const ntm::f32x4*)src, (ntm::f32x4*)dst, n4);
    return (int)hipGetLastError();
  }
  const unsigned g = tiled_grid(n4, unroll, grid);
  switch (unroll) {
    case 2: return copy_u<2>(src, dst, n4, policy, g, S(stream));
    case 4: return copy_u<4>(src, dst, n4, policy, g, S(stream));
    case 8: return copy_u<8>(src, dst, n4, policy, g, S(stream));
    case 16: return copy_u<16>(src, dst, n4, policy, g, S(stream));
    default: return (int)hipErrorInvalidValue;
  }
}

NTM_API int ntm_stream_read_ex(const void* src, size_t bytes, float* sink,
                               int unroll, int policy, int grid, void* stream) {
  if (bytes % 16 || grid < 0) return (int)hipErrorInvalidValue;
  const size_t n4 = bytes / 16;
  if (unroll == 1) {
    hipLaunchKernelGGL(ntm::aux::stream_read_kernel, dim3(2048), dim3(256), 0,
                       S(stream), (const ntm::f32x4*)src, n4, sink);
    return (int)hipGetLastError();
  }
  const unsigned g = tiled_grid(n4, unroll, grid);
  switch (unroll) {
    case 2: return read_u<2>(src, n4, sink, policy, g, S(stream));
    case 4: return read_u<4>(src, n4, sink, policy, g, S(stream));
    case 8: return read_u<8>(src, n4, sink, policy, g, S(stream));
    case 16: return read_u<16>(src, n4, sink, policy, g, S(stream));
    default: return (int)hipErrorInvalidValue;
  }
}

// Tuned defaults (= ops.kernels.STREAM_COPY_CONFIG / STREAM_READ_CONFIG).
// Copy: 2 float4 per lane, nontemporal load + store, one 8 KiB tile per block
// (grid 0): 6.37 TB/s at 2 GiB, 6.05 at 4 GiB against 5.81 / 5.41 for the
// earlier (8, 7, 512) grid-stride pipeline (interleaved, profiles/r2_k2/).
// Read 7.1 TB/s on two MI355X boxes.
NTM_API int ntm_stream_copy(const void* src, void* dst, size_t bytes,
                            void* stream) {
  return ntm_stream_copy_ex(src, dst, bytes, 2, 7, 0, stream);
}

NTM_API int ntm_stream_read(const void* src, size_t bytes, float* sink,
                            void* stream) {
  return ntm_stream_read_ex(src, bytes, sink, 8, 1, 1024, stream);
}
