"""Writes the golden vectors of tests/golden/*.json.

Every vector below is transcribed by hand from the reference's own tests (Flink
2.3-SNAPSHOT at /root/reference, read as text; the reference is Java and cannot be
compiled or run in this container — SURVEY.md §8c).  The citation next to each block
names the file:line it comes from.  Only data is recorded: inputs and the outputs the
reference's assertions expect.

Run:  python tests/golden/make_golden.py   (rewrites the JSON files next to it)
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
WOT = ("flink-streaming-java/src/test/java/org/apache/flink/streaming/runtime/operators/"
       "windowing/WindowOperatorTest.java")


def dump(name, obj):
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(obj, f, indent=1)
        f.write("\n")


# --------------------------------------------------------------------------------------
# Key groups: RocksIncrementalCheckpointRescalingTest.java:66-132
#   assignToKeyGroup(String key, maxParallelism = 10) with a pass-through key selector.
# --------------------------------------------------------------------------------------
dump("key_groups.json", {
    "source": "flink-state-backends/flink-statebackend-rocksdb/src/test/java/org/apache/flink/"
              "state/rocksdb/RocksIncrementalCheckpointRescalingTest.java:66-132",
    "max_parallelism": 10,
    "string_keys": [["8", 0], ["5", 1], ["25", 2], ["13", 3], ["4", 4],
                    ["7", 5], ["1", 6], ["6", 7], ["9", 8], ["3", 9]],
})

# --------------------------------------------------------------------------------------
# TimeWindow.getWindowStartWithOffset: TimeWindowTest.java:32-77  [ts, offset, size, start]
# --------------------------------------------------------------------------------------
TWT = "flink-runtime/src/test/java/org/apache/flink/streaming/runtime/operators/windowing/TimeWindowTest.java"
ws = []
for ts, st in [(-8, -14), (-7, -7), (-6, -7), (-1, -7), (1, 0), (6, 0), (7, 7), (8, 7)]:
    ws.append([ts, 0, 7, st])
for ts, st in [(-10, -11), (-9, -11), (-3, -4), (-2, -4), (-1, -4), (1, -4), (2, -4),
               (3, 3), (9, 3), (10, 10)]:
    ws.append([ts, 3, 7, st])
for ts, st in [(-12, -16), (-7, -9), (-4, -9), (-3, -9), (2, -2), (-1, -2), (1, -2), (-2, -2),
               (3, -2), (4, -2), (7, 5), (12, 12)]:
    ws.append([ts, -2, 7, st])
ws.append([1470902048450, -8 * 3600 * 1000, 24 * 3600 * 1000, 1470844800000])
dump("window_start.json", {"source": TWT + ":32-77", "cases": ws})

# --------------------------------------------------------------------------------------
# Assigners: [assigner, size, slide, offset, ts, [[start, end], ...]]
# --------------------------------------------------------------------------------------
SEW = ("flink-runtime/src/test/java/org/apache/flink/streaming/runtime/operators/windowing/"
       "SlidingEventTimeWindowsTest.java")
TEW = ("flink-runtime/src/test/java/org/apache/flink/streaming/runtime/operators/windowing/"
       "TumblingEventTimeWindowsTest.java")
SES = ("flink-streaming-java/src/test/java/org/apache/flink/streaming/runtime/operators/"
       "windowing/EventTimeSessionWindowsTest.java")
asg = [
    # SlidingEventTimeWindowsTest.java:39-70 (size 5000, slide 1000)
    ["sliding", 5000, 1000, 0, 0, [[-4000, 1000], [-3000, 2000], [-2000, 3000], [-1000, 4000], [0, 5000]]],
    ["sliding", 5000, 1000, 0, 4999, [[0, 5000], [1000, 6000], [2000, 7000], [3000, 8000], [4000, 9000]]],
    ["sliding", 5000, 1000, 0, 5000, [[1000, 6000], [2000, 7000], [3000, 8000], [4000, 9000], [5000, 10000]]],
    # :72-103 (offset 100)
    ["sliding", 5000, 1000, 100, 100, [[-3900, 1100], [-2900, 2100], [-1900, 3100], [-900, 4100], [100, 5100]]],
    ["sliding", 5000, 1000, 100, 5099, [[100, 5100], [1100, 6100], [2100, 7100], [3100, 8100], [4100, 9100]]],
    ["sliding", 5000, 1000, 100, 5100, [[1100, 6100], [2100, 7100], [3100, 8100], [4100, 9100], [5100, 10100]]],
    # :105-135 (offset -100)
    ["sliding", 5000, 1000, -100, 0, [[-4100, 900], [-3100, 1900], [-2100, 2900], [-1100, 3900], [-100, 4900]]],
    ["sliding", 5000, 1000, -100, 4899, [[-100, 4900], [900, 5900], [1900, 6900], [2900, 7900], [3900, 8900]]],
    ["sliding", 5000, 1000, -100, 4900, [[900, 5900], [1900, 6900], [2900, 7900], [3900, 8900], [4900, 9900]]],
    # TumblingEventTimeWindowsTest.java:41-52
    ["tumbling", 5000, 0, 0, 0, [[0, 5000]]],
    ["tumbling", 5000, 0, 0, 4999, [[0, 5000]]],
    ["tumbling", 5000, 0, 0, 5000, [[5000, 10000]]],
    # :70-82 (global offset 100)
    ["tumbling", 5000, 0, 100, 100, [[100, 5100]]],
    ["tumbling", 5000, 0, 100, 5099, [[100, 5100]]],
    ["tumbling", 5000, 0, 100, 5100, [[5100, 10100]]],
    # :84-97 (global offset -100)
    ["tumbling", 5000, 0, -100, 0, [[-100, 4900]]],
    ["tumbling", 5000, 0, -100, 4899, [[-100, 4900]]],
    ["tumbling", 5000, 0, -100, 4900, [[4900, 9900]]],
    # EventTimeSessionWindowsTest.java:53-66 (gap 5000; "size" column carries the gap)
    ["session", 5000, 0, 0, 0, [[0, 5000]]],
    ["session", 5000, 0, 0, 4999, [[4999, 9999]]],
    ["session", 5000, 0, 0, 5000, [[5000, 10000]]],
]
dump("assigners.json", {"source": [SEW + ":39-135", TEW + ":41-97", SES + ":53-66"], "cases": asg})

# TumblingEventTimeWindowsTest.testWindowAssignmentWithStagger (:55-72): NATURAL stagger, size 5000,
# global offset 0, the first element at processing time 150:
#   [stagger, size, global offset, processing time, ts, [[start, end]]]
dump("stagger.json", {"source": TEW + ":55-72", "cases": [
    ["NATURAL", 5000, 0, 150, 150, [[150, 5150]]],
    ["NATURAL", 5000, 0, 150, 5099, [[150, 5150]]],
    ["NATURAL", 5000, 0, 150, 5300, [[5150, 10150]]],
]})

# --------------------------------------------------------------------------------------
# TimeWindow.mergeWindows via EventTimeSessionWindows.mergeWindows:
#   [[input windows], [[merged members...], cover], ...]  (only groups of size > 1)
# --------------------------------------------------------------------------------------
dump("merge_windows.json", {"source": SES + ":68-165", "cases": [
    [[[0, 0]], []],                                   # testMergeSinglePointWindow
    [[[0, 1]], []],                                   # testMergeSingleWindow
    [[[0, 1], [1, 2], [2, 3], [4, 5], [5, 6]],        # testMergeConsecutiveWindows
     [[[[0, 1], [1, 2], [2, 3]], [0, 3]], [[[4, 5], [5, 6]], [4, 6]]]],
    [[[1, 1], [0, 2], [4, 7], [5, 6]],                # testMergeCoveringWindow
     [[[[1, 1], [0, 2]], [0, 2]], [[[5, 6], [4, 7]], [4, 7]]]],
]})

# --------------------------------------------------------------------------------------
# MergingWindowSet driven directly, EventTimeSessionWindows.withGap(3 ms)
# (MergingWindowSetTest.java).  Steps:
#   ["add", window, result, merge]   merge: null (the MergeFunction did not run) or
#       {"target": w, "state_window": [allowed w...], "sources": [w...] (as a set),
#        "merged_state_windows": [[allowed set of w]...] | null (unchecked)}
#   ["state", window, [allowed state windows] | null (getStateWindow == null)]
#   ["retire", window]        ["persist", [[window, state window]...] (as a set)]
# "restore": the ListState the set is constructed from.  Where the reference accepts any of
# several state windows (the first element of a HashSet, MergingWindowSet.java:190) every
# allowed answer is listed.
# --------------------------------------------------------------------------------------
MWST = ("flink-streaming-java/src/test/java/org/apache/flink/streaming/runtime/operators/"
        "windowing/MergingWindowSetTest.java")
W0_4, W3_5, W0_5, W4_6, W0_6 = [0, 4], [3, 5], [0, 5], [4, 6], [0, 6]
mws_tests = [
    {"name": "incremental_merging", "source": MWST + ":90-206", "restore": [], "steps": [
        ["add", W0_4, W0_4, None], ["state", W0_4, [W0_4]],
        ["add", W0_4, W0_4, None],
        ["add", W3_5, W0_5, {"target": W0_5, "state_window": [W0_4], "sources": [W0_4],
                             "merged_state_windows": [[]]}],
        ["add", W4_6, W0_6, {"target": W0_6, "state_window": [W0_4], "sources": [W0_5],
                             "merged_state_windows": [[]]}],
        ["state", W0_6, [W0_4]],
        ["add", [1, 4], W0_6, None], ["add", W0_4, W0_6, None], ["add", W3_5, W0_6, None],
        ["add", W4_6, W0_6, None], ["state", W0_6, [W0_4]],
        ["add", [11, 14], [11, 14], None], ["state", W0_6, [W0_4]], ["state", [11, 14], [[11, 14]]],
        ["add", [10, 13], [10, 14], {"target": [10, 14], "state_window": [[11, 14]], "sources": [[11, 14]],
                                     "merged_state_windows": [[]]}],
        ["add", [12, 15], [10, 15], {"target": [10, 15], "state_window": [[11, 14]], "sources": [[10, 14]],
                                     "merged_state_windows": [[]]}],
        ["add", [11, 14], [10, 15], None],
        ["state", W0_6, [W0_4]], ["state", [10, 15], [[11, 14]]],
        ["retire", W0_6], ["state", W0_6, None], ["state", [10, 15], [[11, 14]]],
    ]},
    {"name": "late_merging", "source": MWST + ":208-303", "restore": [], "steps": [
        ["add", [0, 3], [0, 3], None], ["state", [0, 3], [[0, 3]]],
        ["add", [5, 8], [5, 8], None], ["state", [5, 8], [[5, 8]]],
        ["add", [10, 13], [10, 13], None], ["state", [10, 13], [[10, 13]]],
        ["add", [8, 10], [5, 13], {"target": [5, 13], "state_window": [[5, 8], [10, 13]],
                                   "sources": [[5, 8], [10, 13]],
                                   "merged_state_windows": [[[10, 13]], [[5, 8]]]}],
        ["state", [0, 3], [[0, 3]]],
        ["add", [5, 8], [5, 13], None], ["add", [8, 10], [5, 13], None], ["add", [10, 13], [5, 13], None],
        ["state", [5, 13], [[5, 8], [10, 13]]],
        ["add", [3, 5], [0, 13], {"target": [0, 13], "state_window": [[0, 3], [5, 8], [10, 13]],
                                  "sources": [[0, 3], [5, 13]],
                                  "merged_state_windows": [[[0, 3]], [[5, 8]], [[10, 13]]]}],
        ["state", [0, 13], [[0, 3], [5, 8], [10, 13]]],
    ]},
    {"name": "large_window_covering_single_window", "source": MWST + ":305-332", "restore": [], "steps": [
        ["add", [1, 2], [1, 2], None], ["state", [1, 2], [[1, 2]]],
        ["add", [0, 3], [0, 3], {"target": [0, 3], "state_window": [[1, 2]], "sources": [[1, 2]],
                                 "merged_state_windows": None}],
        ["state", [0, 3], [[1, 2]]],
    ]},
    {"name": "adding_identical_windows", "source": MWST + ":334-360", "restore": [], "steps": [
        ["add", [1, 2], [1, 2], None], ["state", [1, 2], [[1, 2]]],
        ["add", [1, 2], [1, 2], None], ["state", [1, 2], [[1, 2]]],
    ]},
    {"name": "large_window_covering_multiple_windows", "source": MWST + ":362-419", "restore": [], "steps": [
        ["add", [1, 3], [1, 3], None], ["state", [1, 3], [[1, 3]]],
        ["add", [5, 8], [5, 8], None], ["state", [5, 8], [[5, 8]]],
        ["add", [10, 13], [10, 13], None], ["state", [10, 13], [[10, 13]]],
        # transcribed as written (:402-415): the alternatives name (0, 3), which the set never
        # holds (the first window is (1, 3)), so only {(5, 8), (10, 13)} can pass -- the
        # reference's HashSet order makes (1, 3) the state window here, and so must the oracle
        ["add", [0, 13], [0, 13], {"target": [0, 13], "state_window": [[1, 3], [5, 8], [10, 13]],
                                   "sources": [[1, 3], [5, 8], [10, 13]],
                                   "merged_state_windows": [[[0, 3], [5, 8]], [[0, 3], [10, 13]],
                                                            [[5, 8], [10, 13]]]}],
        ["state", [0, 13], [[1, 3], [5, 8], [10, 13]]],
    ]},
    {"name": "restore_from_state", "source": MWST + ":421-438",
     "restore": [[[17, 42], [42, 17]], [[1, 2], [3, 4]]], "steps": [
        ["state", [17, 42], [[42, 17]]], ["state", [1, 2], [[3, 4]]],
    ]},
    {"name": "persist", "source": MWST + ":440-472", "restore": [], "steps": [
        ["add", [1, 2], [1, 2], None], ["add", [17, 42], [17, 42], None],
        ["state", [1, 2], [[1, 2]]], ["state", [17, 42], [[17, 42]]],
        ["persist", [[[1, 2], [1, 2]], [[17, 42], [17, 42]]]],
    ]},
    {"name": "persist_only_if_have_updates", "source": MWST + ":474-495",
     "restore": [[[17, 42], [42, 17]], [[1, 2], [3, 4]]], "steps": [
        ["state", [17, 42], [[42, 17]]], ["state", [1, 2], [[3, 4]]],
        ["persist", [[[1, 2], [3, 4]], [[17, 42], [42, 17]]]],
    ]},
]
dump("merging_window_set.json", {"source": MWST, "gap": 3, "tests": mws_tests})

# --------------------------------------------------------------------------------------
# Operator harness tests (KeyedOneInputStreamOperatorTestHarness, HashMapStateBackend).
# ops: ["e", key, value, ts] | ["w", wm, [expected rows]]
# expected row: [key, result, timestamp(=end-1), start|null, end|null]
# Snapshot/restore points of the reference tests do not change the expected output
# and are recorded as ["snapshot"] markers.
# --------------------------------------------------------------------------------------
common_in = [["e", "key2", 1, 3999], ["e", "key2", 1, 3000], ["e", "key1", 1, 20],
             ["e", "key1", 1, 0], ["e", "key1", 1, 999], ["e", "key2", 1, 1998],
             ["e", "key2", 1, 1999], ["e", "key2", 1, 1000]]
ops_tests = []
# testSlidingEventTimeWindows (:116-219): SlidingEventTimeWindows.of(3s, 1s), SumReducer
ops_tests.append({
    "name": "sliding_3s_1s_sum", "source": WOT + ":116-219",
    "config": {"assigner": "sliding", "size": 3000, "slide": 1000, "agg": "sum_i32"},
    "ops": common_in + [
        ["w", 999, [["key1", 3, 999, None, None]]],
        ["w", 1999, [["key1", 3, 1999, None, None], ["key2", 3, 1999, None, None]]],
        ["w", 2999, [["key1", 3, 2999, None, None], ["key2", 3, 2999, None, None]]],
        ["snapshot"],
        ["w", 3999, [["key2", 5, 3999, None, None]]],
        ["w", 4999, [["key2", 2, 4999, None, None]]],
        ["w", 5999, [["key2", 2, 5999, None, None]]],
        ["w", 6999, []], ["w", 7999, []]],
    "late": 0,
})
# testTumblingEventTimeWindows (:333-434): TumblingEventTimeWindows.of(3s), SumReducer
ops_tests.append({
    "name": "tumbling_3s_sum", "source": WOT + ":333-434",
    "config": {"assigner": "tumbling", "size": 3000, "agg": "sum_i32"},
    "ops": common_in + [
        ["w", 999, []], ["w", 1999, []], ["snapshot"],
        ["w", 2999, [["key1", 3, 2999, None, None], ["key2", 3, 2999, None, None]]],
        ["w", 3999, []], ["w", 4999, []],
        ["w", 5999, [["key2", 2, 5999, None, None]]],
        ["w", 6999, []], ["w", 7999, []]],
    "late": 0,
})
# testSessionWindows (:543-632) and testReduceSessionWindows (:730-816): gap 3s,
# SessionWindowFunction / ReducedSessionWindowFunction emit (key-sum, start, end)@end-1.
sess_ops = [["e", "key2", 1, 0], ["e", "key2", 2, 1000], ["e", "key2", 3, 2500],
            ["e", "key1", 1, 10], ["e", "key1", 2, 1000], ["snapshot"],
            ["e", "key1", 3, 2500], ["e", "key2", 4, 5501], ["e", "key2", 5, 6000],
            ["e", "key2", 5, 6000], ["e", "key2", 6, 6050],
            ["w", 12000, [["key1", 6, 5499, 10, 5500], ["key2", 6, 5499, 0, 5500],
                          ["key2", 20, 9049, 5501, 9050]]],
            ["e", "key2", 10, 15000], ["e", "key2", 20, 15000],
            ["w", 17999, [["key2", 30, 17999, 15000, 18000]]]]
ops_tests.append({"name": "session_3s_sum", "source": WOT + ":543-632",
                  "config": {"assigner": "session", "gap": 3000, "agg": "sum_i32"},
                  "ops": sess_ops, "late": 0})
red_ops = [["e", "key2", 1, 0], ["e", "key2", 2, 1000], ["e", "key2", 3, 2500], ["snapshot"],
           ["e", "key1", 1, 10], ["e", "key1", 2, 1000], ["e", "key1", 3, 2500],
           ["e", "key2", 4, 5501], ["e", "key2", 5, 6000], ["e", "key2", 5, 6000],
           ["e", "key2", 6, 6050],
           ["w", 12000, [["key1", 6, 5499, 10, 5500], ["key2", 6, 5499, 0, 5500],
                         ["key2", 20, 9049, 5501, 9050]]],
           ["e", "key2", 10, 15000], ["e", "key2", 20, 15000],
           ["w", 17999, [["key2", 30, 17999, 15000, 18000]]]]
ops_tests.append({"name": "reduce_session_3s_sum", "source": WOT + ":730-816",
                  "config": {"assigner": "session", "gap": 3000, "agg": "sum_i32"},
                  "ops": red_ops, "late": 0})
# testLateness (:2038-2137): Tumbling 2s, PurgingTrigger(EventTimeTrigger), lateness 500,
# late element 1998 goes to the side output (counted as late_dropped here).
ops_tests.append({
    "name": "lateness_tumbling_2s_purging", "source": WOT + ":2038-2137",
    "config": {"assigner": "tumbling", "size": 2000, "agg": "sum_i32", "lateness": 500,
               "trigger": "purging_event_time"},
    "ops": [["e", "key2", 1, 500], ["w", 1500, []],
            ["e", "key2", 1, 1300], ["w", 2300, [["key2", 2, 1999, None, None]]],
            ["e", "key2", 1, 1997], ["w", 6000, [["key2", 1, 1999, None, None]]],
            ["e", "key2", 1, 1998], ["w", 7000, []]],
    "late": 1,
    "side": [["key2", 1, 1998]],  # lateOutputTag set (:2066-2067), lateExpected (:2118)
})
# testCleanupTimeOverflow (:2139-2248): Tumbling 1000 ms, lateness 2000,
# ts = Long.MAX_VALUE - 1750 -> window [MAX-1807, MAX-807), maxTs = MAX - 808.
MAXL = (1 << 63) - 1
_ts = MAXL - 1750
_start = _ts - (_ts % 1000)
ops_tests.append({
    "name": "cleanup_time_overflow", "source": WOT + ":2139-2248",
    "config": {"assigner": "tumbling", "size": 1000, "agg": "sum_i32", "lateness": 2000},
    "ops": [["e", "key2", 1, _ts], ["w", MAXL - 1500, []],
            ["w", _start + 999, [["key2", 1, _start + 999, None, None]]]],
    "late": 0,
})
# Session windows and allowed lateness (gap 3 s, ReducedSessionWindowFunction emits
# (key-sum, start, end)@end-1).  Rows a late element fires at once (EventTimeTrigger.onElement
# FIRE) are checked at the next watermark with that watermark's rows.
_sl_in = [["e", "key2", 1, 1000], ["w", 1999, []], ["e", "key2", 1, 2000], ["w", 4998, []],
          ["e", "key2", 1, 4500], ["e", "key2", 1, 8500], ["w", 7400, []],
          ["e", "key2", 1, 7000], ["w", 11501, [["key2", 5, 11499, 1000, 11500]]],
          ["e", "key2", 1, 11600], ["w", 14600, [["key2", 1, 14599, 11600, 14600]]]]
# testSideOutputDueToLatenessSessionZeroLateness (:2571-2668): the element at 10000 is late
# (side output; counted as late_dropped here).
ops_tests.append({"name": "session_lateness_zero", "source": WOT + ":2571-2668",
                  "config": {"assigner": "session", "gap": 3000, "agg": "sum_i32"},
                  "ops": _sl_in + [["e", "key2", 1, 10000], ["e", "key2", 1, 14500],
                                   ["w", 20000, [["key2", 1, 17499, 14500, 17500]]], ["w", 100000, []]],
                  "late": 1, "side": [["key2", 1, 10000]]})
# testNotSideOutputDueToLatenessSessionWithLateness (:2766-2879): lateness 10 ms; 10000
# merges into the fired (11600, 14600) session and fires (10000, 14600) at once.
ops_tests.append({"name": "session_lateness_10", "source": WOT + ":2766-2879",
                  "config": {"assigner": "session", "gap": 3000, "agg": "sum_i32", "lateness": 10},
                  "ops": _sl_in + [["e", "key2", 1, 10000], ["e", "key2", 1, 14500],
                                   ["w", 20000, [["key2", 2, 14599, 10000, 14600],
                                                 ["key2", 3, 17499, 10000, 17500]]], ["w", 100000, []]],
                  "late": 0, "side": []})
# testNotSideOutputDueToLatenessSessionWithHugeLateness (:2984-3083): lateness 10 s; the
# fired (1000, 11500) session is still kept, so 10000 merges everything into (1000, 14600).
ops_tests.append({"name": "session_lateness_huge", "source": WOT + ":2984-3083",
                  "config": {"assigner": "session", "gap": 3000, "agg": "sum_i32", "lateness": 10000},
                  "ops": _sl_in + [["e", "key2", 1, 10000], ["e", "key2", 1, 14500],
                                   ["w", 20000, [["key2", 7, 14599, 1000, 14600],
                                                 ["key2", 8, 17499, 1000, 17500]]], ["w", 100000, []]],
                  "late": 0, "side": []})
# testDropDueToLatenessSessionWithLatenessPurgingTrigger (:2670-2765) and
# testNotSideOutputDueToLatenessSessionWithHugeLatenessPurgingTrigger (:2881-2983):
# PurgingTrigger(EventTimeTrigger); a fired session keeps an empty state until cleanup.
for _name, _src, _lat, _start in (("session_lateness_10_purging", ":2670-2765", 10, 10000),
                                  ("session_lateness_huge_purging", ":2881-2983", 10000, 1000)):
    ops_tests.append({"name": _name, "source": WOT + _src,
                      "config": {"assigner": "session", "gap": 3000, "agg": "sum_i32", "lateness": _lat,
                                 "trigger": "purging_event_time"},
                      "ops": _sl_in + [["e", "key2", 1, 10000], ["e", "key2", 1, 14500],
                                       ["w", 20000, [["key2", 1, 14599, _start, 14600],
                                                     ["key2", 1, 17499, _start, 17500]]], ["w", 100000, []]],
                      "late": 0, **({"side": []} if _lat == 10000 else {})})
# Late-data side output (WindowedStream.sideOutputLateData; WindowOperator.java:440-446):
# "side" lists the records the side output holds [key, value, timestamp]; without the side
# output they are counted in numLateRecordsDropped ("late").
# testSideOutputDueToLatenessTumbling (:2249-2346): Tumbling 2 s, lateness 0, SumReducer.
ops_tests.append({
    "name": "side_output_tumbling", "source": WOT + ":2249-2346",
    "config": {"assigner": "tumbling", "size": 2000, "agg": "sum_i32"},
    "ops": [["e", "key2", 1, 1000], ["w", 1985, []],
            ["e", "key2", 1, 1980], ["w", 1999, [["key2", 2, 1999, None, None]]],
            ["e", "key2", 1, 1998], ["e", "key2", 1, 2001], ["w", 2999, []],
            ["w", 3999, [["key2", 1, 3999, None, None]]]],
    "late": 1, "side": [["key2", 1, 1998]],
})
# testSideOutputDueToLatenessSliding (:2348-2462): Sliding 3 s / 1 s, lateness 0; the 2400
# elements still fall into the windows ending at 3999 and 4999 (not skipped).
ops_tests.append({
    "name": "side_output_sliding", "source": WOT + ":2348-2462",
    "config": {"assigner": "sliding", "size": 3000, "slide": 1000, "agg": "sum_i32"},
    "ops": [["e", "key2", 1, 1000], ["w", 1999, [["key2", 1, 1999, None, None]]],
            ["e", "key2", 1, 2000], ["w", 3000, [["key2", 2, 2999, None, None]]],
            ["e", "key1", 1, 3001], ["e", "key2", 1, 2400], ["e", "key2", 1, 2400], ["e", "key1", 1, 3001],
            ["e", "key2", 1, 3900],
            ["w", 6000, [["key2", 5, 3999, None, None], ["key1", 2, 3999, None, None],
                         ["key2", 4, 4999, None, None], ["key1", 2, 4999, None, None],
                         ["key2", 1, 5999, None, None], ["key1", 2, 5999, None, None]]],
            ["e", "key1", 1, 3001], ["w", 25000, []]],
    "late": 1, "side": [["key1", 1, 3001]],
})
# testSideOutputDueToLatenessSessionZeroLatenessPurgingTrigger (:2465-2569): gap 3 s,
# lateness 0, PurgingTrigger(EventTimeTrigger).
ops_tests.append({"name": "side_output_session_zero_lateness_purging", "source": WOT + ":2465-2569",
                  "config": {"assigner": "session", "gap": 3000, "agg": "sum_i32",
                             "trigger": "purging_event_time"},
                  "ops": _sl_in + [["e", "key2", 1, 10000], ["e", "key2", 1, 10100], ["e", "key2", 1, 14500],
                                   ["w", 20000, [["key2", 1, 17499, 14500, 17500]]], ["w", 100000, []]],
                  "late": 2, "side": [["key2", 1, 10000], ["key2", 1, 10100]]})
# SessionWindowing example (flink-examples-streaming SessionWindowing.java:58-69, gap 3 ms
# at :94, sum(2)) with expected output SessionWindowingData.java:23-24.  The tuple's f1
# (first element's timestamp) equals the session start for this input.
EXS = "flink-examples/flink-examples-streaming/src/main/java/org/apache/flink/streaming/examples/windowing/"
ops_tests.append({
    "name": "session_windowing_example", "source": [EXS + "SessionWindowing.java:58-94",
                                                    EXS + "util/SessionWindowingData.java:23-24"],
    "config": {"assigner": "session", "gap": 3, "agg": "sum_i32"},
    "ops": [["e", "a", 1, 1], ["e", "b", 1, 1], ["e", "b", 1, 3], ["e", "b", 1, 5],
            ["e", "c", 1, 6], ["e", "a", 1, 10], ["e", "c", 1, 11],
            ["w", MAXL, [["a", 1, 3, 1, 4], ["c", 1, 8, 6, 9], ["c", 1, 13, 11, 14],
                         ["b", 3, 7, 1, 8], ["a", 1, 12, 10, 13]]]],
    "late": 0,
})
dump("operator_harness.json", {"tests": ops_tests})

# Count windows: EvictingWindowOperatorTest.testCountTrigger (flink-streaming-java/src/test/
# java/org/apache/flink/streaming/runtime/operators/windowing/EvictingWindowOperatorTest.java
# :730-841): GlobalWindows + CountTrigger.of(2) + CountEvictor.of(4) = countWindow(4, 2),
# SumReducer over Tuple2<String, Integer>.f1; every output carries Long.MAX_VALUE.  The
# expected rows are checked as a multiset after each group of elements, as the test does
# (assertOutputEqualsSorted).
EWOT = ("flink-streaming-java/src/test/java/org/apache/flink/streaming/runtime/operators/windowing/"
        "EvictingWindowOperatorTest.java")
dump("count_windows.json", {"tests": [{
    "name": "count_trigger_count_evictor", "source": EWOT + ":730-841",
    "config": {"assigner": "count_sliding", "size": 4, "slide": 2, "agg": "sum_i32"},
    "groups": [
        {"elements": [["key2", 1], ["key2", 1], ["key1", 1], ["key1", 1], ["key1", 1],
                      ["key2", 1], ["key2", 1], ["key2", 1]],
         "expected": [["key2", 2], ["key2", 4], ["key1", 2]]},
        {"elements": [["key1", 1], ["key2", 1]],
         "expected": [["key1", 4], ["key2", 4]]},
    ],
}]})

# --------------------------------------------------------------------------------------
# minBy / maxBy: AggregationFunctionTest.minMaxByTest (flink-runtime/src/test/java/org/apache/
# flink/streaming/api/AggregationFunctionTest.java:227-345; input getInputByList :491-497).
# Tuple3(0, i % 3, i) for i in 0..8, keyed by f0, ComparableAggregator(1, MAXBY / MINBY,
# first) reduced by StreamGroupedReduceOperator: one output per element, the running element.
# As windows: after element p the row of a window holding elements 0..p stands for expected[p].
# --------------------------------------------------------------------------------------
AFT = "flink-runtime/src/test/java/org/apache/flink/streaming/api/AggregationFunctionTest.java"
dump("minmaxby.json", {
    "source": AFT + ":227-345",
    "input": [[0, i % 3, i] for i in range(9)],
    "by_field": 1,
    "expected": {
        "maxBy_first": [[0, 0, 0], [0, 1, 1], [0, 2, 2], [0, 2, 2], [0, 2, 2], [0, 2, 2], [0, 2, 2], [0, 2, 2],
                        [0, 2, 2]],
        "maxBy_last": [[0, 0, 0], [0, 1, 1], [0, 2, 2], [0, 2, 2], [0, 2, 2], [0, 2, 5], [0, 2, 5], [0, 2, 5],
                       [0, 2, 8]],
        "minBy_first": [[0, 0, 0]] * 9,
        "minBy_last": [[0, 0, 0], [0, 0, 0], [0, 0, 0], [0, 0, 3], [0, 0, 3], [0, 0, 3], [0, 0, 6], [0, 0, 6],
                       [0, 0, 6]],
    },
})

print("golden vectors written to", HERE)
