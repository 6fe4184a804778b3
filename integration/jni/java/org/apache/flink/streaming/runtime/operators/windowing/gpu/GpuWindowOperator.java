/*
 * GpuWindowOperator — drop-in for WindowOperator on the keyed event-time aggregation path,
 * backed by libgpuwin.so (MI355X).  NOT BUILT in this repository (no JDK in the build image);
 * it shows the reference-side binding a Flink maintainer adds.  It fills the same slot as
 * WindowOperator (flink-runtime/.../operators/windowing/WindowOperator.java:102): a
 * OneInputStreamOperator inserted by WindowedStream via input.transform(...)
 * (WindowedStream.java:233-240, DataStream.java:815-821).
 *
 * Records between two watermarks are appended to off-heap columns; processWatermark hands
 * the batch to the GPU, advances event time, and emits the fired rows BEFORE forwarding the
 * watermark, as AbstractStreamOperator.processWatermark does (AbstractStreamOperator.java:
 * 690-703).  Count windows fire on the element (CountTrigger.onElement), so their rows are
 * emitted right after each batch is handed over.
 *
 * Output (OutputMode), with the record timestamp window.maxTimestamp() = end - 1
 * (WindowOperator.emitWindowContents :575-580):
 *   POSITIONAL     WindowedStream.sum/min/max(i): the window's first element (arrival order)
 *                  with field i replaced by the result -- SumAggregator / ComparableAggregator
 *                  keep the first element's other fields (SumAggregator.java:66-76,
 *                  ComparableAggregator.java:83-104).  Tuple2<Long, X>: (key, result).  Wider
 *                  tuples: the handle runs with GW_FLAG_FIRST_ELEMENT, each element's payload is
 *                  its arrival sequence, the elements wait in an ElementLog until no window can
 *                  reach them, and each row's payload picks its first element.
 *   MIN_MAX_BY     WindowedStream.minBy/maxBy(i, first) (WindowedStream.java:725-771): the
 *                  element itself whose field i is the window's minimum / maximum, the first of
 *                  equal ones or the last (ComparableAggregator.java:88-95); agg is GW_MIN_* /
 *                  GW_MAX_*, the handle runs with GW_FLAG_BY_FIELD (+ GW_FLAG_BY_LAST), payloads
 *                  and the ElementLog as for wide POSITIONAL rows.
 *   AGGREGATE      WindowedStream.aggregate(AggregateFunction): getResult(acc) alone (Long for
 *                  count, Double for avg), PassThroughWindowFunction.
 *   KEYED_WINDOW   Tuple4 (key, window start, window end, result), what a ProcessWindowFunction
 *                  emitting (key, window, result) produces.
 *   WINDOW_FUNCTION the user's window function over the pre-aggregated result:
 *                  reduce(ReduceFunction, ProcessWindowFunction | WindowFunction) and
 *                  aggregate(AggregateFunction, ProcessWindowFunction | WindowFunction)
 *                  (WindowedStream.java:224-276, 342-526).  As InternalSingleValueProcessWindowFunction
 *                  does, the function gets the key, the window and a one-element Iterable of the
 *                  GPU's result, and emits through a collector stamped window.maxTimestamp().
 *                  Per-window / global keyed state of the Context is not available
 *                  (UnsupportedOperationException).
 *
 * Aggregates: the closed set of gw_agg (count, sum, min, max, avg over Long / Double fields).
 * A job whose AggregateFunction / ReduceFunction is anything else keeps the reference
 * WindowOperator: it cannot be expressed as a gw_agg, and no GpuWindowOperator is created for it.
 *
 * Stagger (TumblingEventTimeWindows.of(size, offset, WindowStagger)): the stagger offset is
 * drawn at the first element, as TumblingEventTimeWindows.assignWindows does
 * (TumblingEventTimeWindows.java:72-79), so a staggered operator creates its handle then, with
 * offset (offset + stagger) % size (gw_window_stagger_offset).  A staggered operator restored
 * from window state reuses the stagger the state was written under (the blob's window offset):
 * the reference would draw a new one and keep the restored windows' alignment beside it, which
 * one handle cannot hold; for RANDOM the old draw is a valid draw.  Restored key groups drawn
 * with different staggers are refused.
 *
 * Keys (K, as WindowOperator<K, ...> at WindowOperator.java:102): Long keys go to the GPU as
 * they are, and the device computes Long.hashCode.  Any other key type (String, Integer,
 * POJOs) gets an int64 id from a KeyDictionary, and key.hashCode() travels in the keyHashes
 * column: key groups, snapshots and rescaling follow the key's own hash
 * (KeyGroupRangeAssignment.java:63-66), and GW_FLAG_CHECK_KEY_GROUPS verifies every batch
 * against this subtask's key-group range.  Snapshots write the blob per key group, then each
 * key its entries name through the key serializer; a restore maps those keys to this
 * subtask's ids (gw_snapshot_remap_keys) before gw_restore.
 */
package org.apache.flink.streaming.runtime.operators.windowing.gpu;

import org.apache.flink.api.common.externalresource.ExternalResourceInfo;
import org.apache.flink.api.common.functions.DefaultOpenContext;
import org.apache.flink.api.common.functions.util.FunctionUtils;
import org.apache.flink.api.common.state.KeyedStateStore;
import org.apache.flink.streaming.api.functions.windowing.ProcessWindowFunction;
import org.apache.flink.streaming.api.functions.windowing.WindowFunction;
import org.apache.flink.streaming.api.operators.TimestampedCollector;
import org.apache.flink.streaming.api.windowing.assigners.WindowStagger;
import org.apache.flink.streaming.api.windowing.windows.TimeWindow;
import org.apache.flink.util.Collector;
import org.apache.flink.api.java.functions.KeySelector;
import org.apache.flink.api.java.tuple.Tuple;
import org.apache.flink.api.java.tuple.Tuple2;
import org.apache.flink.api.java.tuple.Tuple4;
import org.apache.flink.runtime.state.KeyGroupRange;
import org.apache.flink.runtime.state.KeyGroupStatePartitionStreamProvider;
import org.apache.flink.runtime.state.KeyedStateCheckpointOutputStream;
import org.apache.flink.runtime.state.StateInitializationContext;
import org.apache.flink.runtime.state.StateSnapshotContext;
import org.apache.flink.streaming.api.operators.AbstractStreamOperator;
import org.apache.flink.streaming.api.operators.BoundedOneInput;
import org.apache.flink.streaming.api.operators.OneInputStreamOperator;
import org.apache.flink.streaming.api.watermark.Watermark;
import org.apache.flink.streaming.runtime.streamrecord.StreamRecord;
import org.apache.flink.streaming.runtime.tasks.KeyContextHandler;
import org.apache.flink.util.OutputTag;

import java.io.DataInputStream;
import java.io.DataOutputStream;
import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.ArrayDeque;
import java.util.ArrayList;
import java.util.Collections;
import java.util.HashMap;
import java.util.List;
import java.util.Map;
import java.util.concurrent.ThreadLocalRandom;

import org.apache.flink.api.common.typeutils.TypeSerializer;
import org.apache.flink.core.memory.DataInputViewStreamWrapper;
import org.apache.flink.core.memory.DataOutputViewStreamWrapper;
import java.util.function.ToDoubleFunction;
import java.util.function.ToLongFunction;

public class GpuWindowOperator<IN, K>
        extends AbstractStreamOperator<Object>
        implements OneInputStreamOperator<IN, Object>, BoundedOneInput, KeyContextHandler {

    static { System.loadLibrary("gpuwin_jni"); }

    /** What one fired (key, window, result) row becomes (see the class comment). */
    public enum OutputMode { POSITIONAL, MIN_MAX_BY, AGGREGATE, KEYED_WINDOW, WINDOW_FUNCTION }

    // gw_assigner / gw_trigger / gw_agg codes of include/gpuwin.h
    private static final int GW_COUNT_TUMBLING = 3, GW_COUNT_SLIDING = 4;
    private final int assigner, trigger, agg;
    private final OutputMode mode;
    private final long size, slide, offset, gap, lateness;
    private final KeySelector<IN, K> keySelector;
    private final ToLongFunction<IN> longValue;       // for integer aggregates
    private final ToDoubleFunction<IN> doubleValue;   // for f64 aggregates
    private final int batchCapacity;
    private final int inputArity, positionalField;
    private TypeSerializer<IN> inputSerializer;  // Tuple3+ positional: writes the first elements of a snapshot
    private boolean byFirst = true;              // MIN_MAX_BY: the first of equal elements
    private WindowStagger stagger = WindowStagger.ALIGNED;  // tumbling only
    private ProcessWindowFunction<Object, Object, K, TimeWindow> windowFunction;  // WINDOW_FUNCTION

    private transient long handle;
    private transient ByteBuffer keys, keyHashes, ts, values, oKey, oStart, oEnd, oRes;
    private transient int n;
    private transient List<byte[]> restored;  // per-key-group blobs read in initializeState
    private transient List<Map<Long, K>> restoredKeys;  // their key tables (non-Long keys)
    private transient List<Map<Long, IN>> restoredElements;  // their first elements (Tuple3+ positional)
    private transient KeyDictionary<K> dict;  // null while every key so far is a Long
    private transient boolean longKeys;       // decided by the first key
    private transient boolean keyModeKnown;
    private OutputTag<Tuple2<Object, Object>> lateDataTag;  // sideOutputLateData (null: count and drop)
    private transient ByteBuffer lKey, lTs, lVal;
    // positional on Tuple3+: payload column (arrival sequence), the elements by sequence, and
    // per batch (sequence end, max timestamp) for releasing them
    private transient ByteBuffer payload, oPay;
    private transient ElementLog<IN> elements;
    private transient ArrayDeque<long[]> batches;
    private transient long batchMaxTs;
    private transient int createFlags;            // gw_config.flags, decided in open()
    private transient boolean handleDeferred;     // staggered: the handle comes with the first element
    private transient long deferredWatermark = Long.MIN_VALUE;
    private transient TimestampedCollector<Object> collector;
    private transient WindowContext windowContext;
    private transient long currentWm = Long.MIN_VALUE;  // the watermark the current firing runs at
    private transient boolean staged;  // the column buffers are the library's pinned slots (gw_stage_*)
    private transient int slot;        // the slot processElement fills

    /** inputArity: fields of the input Tuple; positionalField: the aggregated field of a
     *  POSITIONAL sum/min/max (the result replaces it in the emitted tuple). */
    public GpuWindowOperator(int assigner, long size, long slide, long offset, long gap, long lateness,
                             int trigger, int agg, KeySelector<IN, K> keySelector,
                             ToLongFunction<IN> longValue, ToDoubleFunction<IN> doubleValue, int batchCapacity,
                             OutputMode mode, int inputArity, int positionalField) {
        if ((mode == OutputMode.POSITIONAL && inputArity > 2 || mode == OutputMode.MIN_MAX_BY)
                && (assigner > 1 /* tumbling, sliding */ || trigger != 0 /* EventTimeTrigger */)) {
            throw new IllegalArgumentException(
                    "positional sum/min/max on Tuple3+ runs on tumbling / sliding event-time windows with "
                            + "EventTimeTrigger (GW_FLAG_FIRST_ELEMENT); use aggregate(...) otherwise");
        }
        this.inputArity = inputArity;
        this.positionalField = positionalField;
        this.assigner = assigner; this.size = size; this.slide = slide; this.offset = offset;
        this.gap = gap; this.lateness = lateness; this.trigger = trigger; this.agg = agg;
        this.keySelector = keySelector; this.longValue = longValue; this.doubleValue = doubleValue;
        this.batchCapacity = batchCapacity; this.mode = mode;
    }

    /** The input type's serializer (TypeInformation.createSerializer): a Tuple3+ positional
     *  operator writes each window's first element with it when it checkpoints. */
    public GpuWindowOperator<IN, K> withInputSerializer(TypeSerializer<IN> serializer) {
        this.inputSerializer = serializer;
        return this;
    }

    /** minBy / maxBy(i, first): false picks the last of equal elements (GW_FLAG_BY_LAST). */
    public GpuWindowOperator<IN, K> withByFirst(boolean first) {
        this.byFirst = first;
        return this;
    }

    /** TumblingEventTimeWindows.of(size, offset, stagger): the stagger offset is drawn at the
     *  first element (TumblingEventTimeWindows.java:72-79). */
    public GpuWindowOperator<IN, K> withStagger(WindowStagger stagger) {
        if (stagger != WindowStagger.ALIGNED && assigner != 0 /* tumbling */) {
            throw new IllegalArgumentException("WindowStagger applies to TumblingEventTimeWindows only");
        }
        this.stagger = stagger;
        return this;
    }

    /** reduce / aggregate(..., ProcessWindowFunction): the function sees the key, the window and
     *  the GPU's pre-aggregated result (OutputMode.WINDOW_FUNCTION). */
    @SuppressWarnings("unchecked")
    public GpuWindowOperator<IN, K> withWindowFunction(ProcessWindowFunction<?, ?, K, TimeWindow> fn) {
        if (mode != OutputMode.WINDOW_FUNCTION) {
            throw new IllegalArgumentException("a window function needs OutputMode.WINDOW_FUNCTION");
        }
        this.windowFunction = (ProcessWindowFunction<Object, Object, K, TimeWindow>) fn;
        return this;
    }

    /** reduce / aggregate(..., WindowFunction): the legacy apply() form, wrapped like
     *  InternalSingleValueWindowFunction wraps it. */
    @SuppressWarnings("unchecked")
    public GpuWindowOperator<IN, K> withWindowFunction(WindowFunction<?, ?, K, TimeWindow> fn) {
        final WindowFunction<Object, Object, K, TimeWindow> wf = (WindowFunction<Object, Object, K, TimeWindow>) fn;
        return withWindowFunction(new ProcessWindowFunction<Object, Object, K, TimeWindow>() {
            @Override
            public void process(K key, Context ctx, Iterable<Object> in, Collector<Object> out) throws Exception {
                wf.apply(key, ctx.window(), in, out);
            }
        });
    }

    /** WindowedStream.sideOutputLateData (WindowOperator.java:440-446, 587-588) for a Tuple2<Long, X>
     *  input: skipped late elements come back as (key, value) with their timestamp. */
    public GpuWindowOperator<IN, K> withLateDataOutput(OutputTag<Tuple2<Object, Object>> tag) {
        this.lateDataTag = tag;
        return this;
    }

    @Override
    public boolean hasKeyContext() { return false; }  // no per-record setCurrentKey (RecordProcessorUtils.java:47-57)

    @Override
    public void open() throws Exception {
        super.open();
        int parallelism = getRuntimeContext().getTaskInfo().getNumberOfParallelSubtasks();
        createFlags = (lateDataTag != null ? 64 /* GW_FLAG_LATE_SIDE_OUTPUT */ : 0)
                | (mode == OutputMode.MIN_MAX_BY ? 512 /* GW_FLAG_BY_FIELD */ | (byFirst ? 0 : 1024 /* GW_FLAG_BY_LAST */)
                        : wide() ? 128 /* GW_FLAG_FIRST_ELEMENT */ : 0)
                | (parallelism > 1 ? 4 /* GW_FLAG_CHECK_KEY_GROUPS: a foreign key fails the batch */ : 0);
        if (mode == OutputMode.WINDOW_FUNCTION) {
            if (windowFunction == null) throw new IllegalStateException("OutputMode.WINDOW_FUNCTION without withWindowFunction(...)");
            FunctionUtils.setFunctionRuntimeContext(windowFunction, getRuntimeContext());
            FunctionUtils.openFunction(windowFunction, DefaultOpenContext.INSTANCE);
            collector = new TimestampedCollector<>(output);
            windowContext = new WindowContext();
        }
        handleDeferred = stagger != WindowStagger.ALIGNED;
        if (handleDeferred && restored != null && !restored.isEmpty()) {
            // Restored window state keeps the stagger it was written under (the blob header's
            // window offset): the reference draws a new stagger after a restore and keeps the
            // restored windows at their old alignment beside it (TumblingEventTimeWindows.java:
            // 53,72-79); one handle holds one alignment, so the old draw is reused.
            long drawn = restoredWindowOffset(restored);
            if (drawn != Long.MIN_VALUE) {
                createHandle(drawn);
                handleDeferred = false;
            }
        }
        if (!handleDeferred && handle == 0) createHandle(offset);
        if (lateDataTag != null) { lKey = direct(8); lTs = direct(8); lVal = direct(8); }
        if (wide() && inputSerializer == null && getExecutionConfig() != null
                && getContainingTask().getConfiguration().isCheckpointingEnabled()) {
            throw new IllegalStateException("positional sum/min/max on Tuple3+ with checkpointing needs "
                    + "withInputSerializer(...): the snapshot writes each window's first element");
        }
        if (wide()) {
            payload = direct(8); oPay = direct(8);
            elements = new ElementLog<>();
            batches = new ArrayDeque<>();
            batchMaxTs = Long.MIN_VALUE;
        }
        keys = direct(8); keyHashes = direct(4); ts = direct(8); values = direct(8);
        oKey = direct(8); oStart = direct(8); oEnd = direct(8); oRes = direct(8);
        if (!handleDeferred) bindStaging();
        if (restored != null && handleDeferred) restored = null;  // staggered: the blobs hold no window state
        if (restored != null) {  // initializeState runs before open (StreamOperator.java:139)
            for (int i = 0; i < restored.size(); i++) {
                byte[] blob = restored.get(i);
                Map<Long, K> table = restoredKeys.get(i);
                if (table != null) {  // the blob's key ids -> this subtask's dictionary ids
                    long[] from = nativeSnapshotKeys(blob);
                    long[] to = new long[from.length];
                    for (int j = 0; j < from.length; j++) {
                        K key = table.get(from[j]);
                        if (key == null) {
                            throw new IllegalStateException("restored window state names key id " + from[j]
                                    + " that its key table does not hold: corrupt checkpoint");
                        }
                        to[j] = dictionary().idOf(key);
                    }
                    nativeRemapKeys(blob, from, to);
                }
                Map<Long, IN> firsts = restoredElements.get(i);
                if (firsts != null) {  // the first elements join this subtask's ElementLog
                    long[] maxEnd = new long[1];
                    long[] from = nativeSnapshotPayloads(blob, maxEnd);
                    long[] to = new long[from.length];
                    for (int j = 0; j < from.length; j++) {
                        IN first = firsts.get(from[j]);
                        if (first == null) {
                            throw new IllegalStateException("restored window state names element " + from[j]
                                    + " that the checkpoint does not hold: corrupt checkpoint");
                        }
                        to[j] = elements.append(first);
                    }
                    nativeRemapPayloads(blob, from, to);
                    // kept until the latest restored window is cleaned: maxTs + size - 1 = its end - 1
                    batches.addLast(new long[] {elements.end(), maxEnd[0] - size});
                }
                nativeRestore(handle, blob);
            }
            restored = null;
            restoredKeys = null;
            restoredElements = null;
        }
    }

    /** Two library-owned pinned slots (gw_stage_alloc) as the operator's column buffers:
     *  processElement writes each record into the memory the PCIe transfer reads, and the
     *  transfer of one batch overlaps the GPU work of the previous one.  Composite and
     *  first-element handles keep their own direct buffers (nativeIngest / nativeIngestPayload). */
    private void bindStaging() {
        staged = !wide() && nativeStageAlloc(handle, 2, batchCapacity) == 0;
        if (staged) bindSlot(0);
    }

    private void bindSlot(int s) {
        slot = s;
        keys = nativeStageColumn(handle, s, 0, batchCapacity).order(ByteOrder.nativeOrder());
        keyHashes = nativeStageColumn(handle, s, 1, batchCapacity).order(ByteOrder.nativeOrder());
        ts = nativeStageColumn(handle, s, 2, batchCapacity).order(ByteOrder.nativeOrder());
        values = nativeStageColumn(handle, s, 3, batchCapacity).order(ByteOrder.nativeOrder());
    }

    /** The window offset restored state of a staggered operator was written under, or
     *  Long.MIN_VALUE when no blob holds window state (the stagger is then drawn at the first
     *  element).  Blob header (include/gpuwin.h gw_snapshot, little-endian): window offset at
     *  byte 32, key-group range at 60 / 64, payload bytes at 88; a key group without state
     *  is 12 bytes (no entries, no merging window set, no timers). */
    static long restoredWindowOffset(List<byte[]> blobs) {
        long found = Long.MIN_VALUE;
        for (byte[] b : blobs) {
            ByteBuffer h = ByteBuffer.wrap(b).order(ByteOrder.LITTLE_ENDIAN);
            long nk = (long) h.getInt(64) - h.getInt(60) + 1;
            if (h.getLong(88) <= 12 * nk) continue;
            long off = h.getLong(32);
            if (found != Long.MIN_VALUE && found != off) {
                throw new UnsupportedOperationException("restoring window state of staggered tumbling operators "
                        + "drawn with different staggers (window offsets " + found + ", " + off + ") into one");
            }
            found = off;
        }
        return found;
    }

    /** The handle, with the windows' offset (the stagger decided by the caller). */
    private void createHandle(long windowOffset) {
        int subtask = getRuntimeContext().getTaskInfo().getIndexOfThisSubtask();
        int parallelism = getRuntimeContext().getTaskInfo().getNumberOfParallelSubtasks();
        int maxP = getRuntimeContext().getTaskInfo().getMaxNumberOfParallelSubtasks();
        handle = nativeCreate(assigner, trigger, size, slide, windowOffset, gap, lateness, agg, maxP, parallelism,
                              subtask, gpuIndex(), createFlags, 1L << 24, batchCapacity);
    }

    /** A staggered operator's first element: draw the stagger (WindowStagger.getStaggerOffset at
     *  the current processing time), create the handle, replay the watermark seen so far. */
    private void createStaggeredHandle() {
        long now = getProcessingTimeService().getCurrentProcessingTime();
        int code = stagger == WindowStagger.RANDOM ? 1 : stagger == WindowStagger.NATURAL ? 2 : 0;
        createHandle(nativeStaggerOffset(code, now, ThreadLocalRandom.current().nextDouble(), size, offset));
        handleDeferred = false;
        bindStaging();
        if (deferredWatermark != Long.MIN_VALUE) nativeAdvanceWatermark(handle, deferredWatermark);  // no state: fires nothing
    }

    private KeyDictionary<K> dictionary() {
        if (dict == null) {
            dict = new KeyDictionary<>();
            longKeys = false;
            keyModeKnown = true;
        }
        return dict;
    }

    /** The GPU this subtask was given: the "index" property of the first "gpu" external
     *  resource (GPUDriver with integration/gpu-discovery/amd-gpu-discovery.sh), else 0. */
    private int gpuIndex() {
        for (ExternalResourceInfo info : getRuntimeContext().getExternalResourceInfos("gpu")) {
            return info.getProperty("index").map(Integer::parseInt).orElse(0);
        }
        return 0;
    }

    // ---- checkpointing: raw keyed state, one blob per key group -------------------------
    // (the heap backend also writes per key group: HeapSnapshotStrategy.java:97-154)

    @Override
    public void prepareSnapshotPreBarrier(long checkpointId) throws Exception {
        flush();
        nativeFlush(handle);  // buffered records into the window state
    }

    @Override
    public void snapshotState(StateSnapshotContext context) throws Exception {
        super.snapshotState(context);
        KeyGroupRange range = getKeyedStateBackend().getKeyGroupRange();
        if (handleDeferred) {  // staggered, no element yet: no window state (an empty blob per key group)
            KeyedStateCheckpointOutputStream out = context.getRawKeyedOperatorStateOutput();
            for (int kg : range) {
                out.startNewKeyGroup(kg);
                DataOutputStream dos = new DataOutputStream(out);
                dos.writeInt(0);
                dos.writeBoolean(false);
                dos.writeInt(0);
                dos.writeInt(0);
                dos.flush();
            }
            return;
        }
        byte[] all = nativeSnapshot(handle, range.getStartKeyGroup(), range.getEndKeyGroup());
        KeyedStateCheckpointOutputStream out = context.getRawKeyedOperatorStateOutput();
        @SuppressWarnings("unchecked")
        TypeSerializer<K> keySer = (TypeSerializer<K>) getKeyedStateBackend().getKeySerializer();
        for (int kg : range) {
            out.startNewKeyGroup(kg);
            byte[] part = nativeSliceKeyGroup(all, kg);
            DataOutputStream dos = new DataOutputStream(out);
            dos.writeInt(part.length);
            dos.write(part);
            // the keys behind the ids, through the key serializer (none for Long keys)
            long[] ids = dict != null ? nativeSnapshotKeys(part) : new long[0];
            dos.writeBoolean(dict != null);
            dos.writeInt(ids.length);
            DataOutputViewStreamWrapper view = new DataOutputViewStreamWrapper(dos);
            for (long id : ids) {
                dos.writeLong(id);
                keySer.serialize(dict.keyOf(id), view);
            }
            // Tuple3+ positional: each window's first element (the reduced Tuple's other fields)
            long[] firsts = wide() ? nativeSnapshotPayloads(part, new long[1]) : new long[0];
            dos.writeInt(firsts.length);
            for (long seq : firsts) {
                dos.writeLong(seq);
                inputSerializer.serialize(elements.get(seq), view);
            }
            dos.flush();
        }
    }

    @Override
    public void initializeState(StateInitializationContext context) throws Exception {
        super.initializeState(context);
        if (!context.isRestored()) return;
        restored = new ArrayList<>();
        restoredKeys = new ArrayList<>();
        restoredElements = new ArrayList<>();
        @SuppressWarnings("unchecked")
        TypeSerializer<K> keySer = (TypeSerializer<K>) getKeyedStateBackend().getKeySerializer();
        for (KeyGroupStatePartitionStreamProvider p : context.getRawKeyedStateInputs()) {
            DataInputStream in = new DataInputStream(p.getStream());
            byte[] blob = new byte[in.readInt()];
            in.readFully(blob);
            if (blob.length == 0) continue;  // written by a staggered operator before its first element
            restored.add(blob);
            boolean keyed = in.readBoolean();
            int nk = in.readInt();
            Map<Long, K> table = keyed ? new HashMap<>() : null;
            DataInputViewStreamWrapper view = new DataInputViewStreamWrapper(in);
            for (int j = 0; j < nk; j++) {
                long id = in.readLong();
                table.put(id, keySer.deserialize(view));
            }
            restoredKeys.add(table);
            int ne = in.readInt();
            Map<Long, IN> firsts = ne > 0 ? new HashMap<>() : null;
            for (int j = 0; j < ne; j++) {
                long seq = in.readLong();
                firsts.put(seq, inputSerializer.deserialize(view));
            }
            restoredElements.add(firsts);
        }
    }

    private ByteBuffer direct(int width) {
        return ByteBuffer.allocateDirect(batchCapacity * width).order(ByteOrder.nativeOrder());
    }

    @Override
    public void processElement(StreamRecord<IN> element) throws Exception {
        if (handleDeferred) createStaggeredHandle();
        IN v = element.getValue();
        K k = keySelector.getKey(v);
        if (!keyModeKnown) {
            longKeys = k instanceof Long;
            keyModeKnown = true;
        }
        if (longKeys) {
            keys.putLong(n * 8, (Long) k);   // key group = murmur(Long.hashCode(k)), computed on the GPU
        } else {
            keys.putLong(n * 8, dictionary().idOf(k));
            keyHashes.putInt(n * 4, k.hashCode());  // KeyGroupRangeAssignment.assignToKeyGroup(key, ..)
        }
        ts.putLong(n * 8, element.getTimestamp());
        if (doubleValue != null) values.putDouble(n * 8, doubleValue.applyAsDouble(v));
        else if (longValue != null) values.putLong(n * 8, longValue.applyAsLong(v));
        if (wide()) {
            payload.putLong(n * 8, elements.append(v));
            batchMaxTs = Math.max(batchMaxTs, element.getTimestamp());
        }
        if (++n == batchCapacity) flush();
    }

    private boolean wide() { return mode == OutputMode.POSITIONAL && inputArity > 2 || mode == OutputMode.MIN_MAX_BY; }

    /** The first element with the aggregated field replaced by the result, in the field's own type. */
    private Object positionalRow(IN first, Object res) {
        Tuple t = ((Tuple) first).copy();
        Object f = t.getField(positionalField);
        if (f instanceof Integer) res = (int) (long) (Long) res;
        else if (f instanceof Short) res = (short) (long) (Long) res;
        else if (f instanceof Byte) res = (byte) (long) (Long) res;
        else if (f instanceof Float) res = (float) (double) (Double) res;
        t.setField(res, positionalField);
        return t;
    }

    private void flush() {
        // Long keys: no key hash column, the GPU computes Long.hashCode; others: ids + hashCode()
        ByteBuffer kh = longKeys ? null : keyHashes;
        if (n > 0 && wide()) {
            nativeIngestPayload(handle, n, keys, kh, ts, values, payload);
            batches.addLast(new long[] {elements.end(), batchMaxTs});
            batchMaxTs = Long.MIN_VALUE;
        } else if (n > 0 && staged) {
            nativeIngestStage(handle, slot, n, (doubleValue != null || longValue != null ? 1 /* GW_STAGE_VALUE */ : 0)
                    | (longKeys ? 0 : 2 /* GW_STAGE_KEY_HASH */));
            bindSlot(slot ^ 1);  // the other slot, once its previous transfer has read it
        } else if (n > 0) {
            nativeIngest(handle, n, keys, kh, ts, values);
        }
        n = 0;
        if (lateDataTag != null) emitLate();
        // CountTrigger fires on the element: count-window rows exist right after the batch
        if (assigner == GW_COUNT_TUMBLING || assigner == GW_COUNT_SLIDING) emitRows();
    }

    private void emitRows() {
        int got;
        while ((got = wide() ? nativeDrainPayload(handle, oKey, oStart, oEnd, oRes, oPay, batchCapacity)
                             : nativeDrain(handle, oKey, oStart, oEnd, oRes, batchCapacity)) > 0) {
            for (int i = 0; i < got; i++) {
                long end = oEnd.getLong(i * 8);
                Object key = key(oKey.getLong(i * 8));
                Object res = agg == 2 || agg >= 5 && agg <= 8 ? (Object) oRes.getDouble(i * 8) : oRes.getLong(i * 8);
                Object row;
                switch (mode) {
                    case POSITIONAL:
                        row = wide() ? positionalRow(elements.get(oPay.getLong(i * 8)), res) : Tuple2.of(key, res);
                        break;
                    case MIN_MAX_BY: row = elements.get(oPay.getLong(i * 8)); break;
                    case AGGREGATE: row = res; break;
                    case WINDOW_FUNCTION:
                        emitThroughWindowFunction(key, oStart.getLong(i * 8), end, res);
                        continue;
                    default: row = Tuple4.of(key, oStart.getLong(i * 8), end, res);
                }
                // count windows: GlobalWindow.maxTimestamp() = Long.MAX_VALUE
                long tsOut = assigner == GW_COUNT_TUMBLING || assigner == GW_COUNT_SLIDING ? Long.MAX_VALUE : end - 1;
                output.collect(new StreamRecord<>(row, tsOut));
            }
            if (got < batchCapacity) break;
        }
    }

    /** InternalSingleValueProcessWindowFunction.process: the window function over the one
     *  pre-aggregated value, output stamped window.maxTimestamp(); with allowed lateness 0 the
     *  firing also cleans the window up (WindowOperator.clearAllState -> userFunction.clear). */
    @SuppressWarnings("unchecked")
    private void emitThroughWindowFunction(Object key, long start, long end, Object res) throws Exception {
        windowContext.window = new TimeWindow(start, end);
        collector.setAbsoluteTimestamp(end - 1);
        windowFunction.process((K) key, windowContext, Collections.singletonList(res), collector);
        if (lateness == 0) windowFunction.clear(windowContext);
    }

    /** ProcessWindowFunction.Context of a GPU-fired window. */
    private final class WindowContext extends ProcessWindowFunction<Object, Object, K, TimeWindow>.Context {
        TimeWindow window;

        WindowContext() { windowFunction.super(); }

        @Override
        public TimeWindow window() { return window; }

        @Override
        public long currentProcessingTime() { return getProcessingTimeService().getCurrentProcessingTime(); }

        @Override
        public long currentWatermark() { return currentWm; }

        @Override
        public KeyedStateStore windowState() {
            throw new UnsupportedOperationException("per-window state in a GPU window function");
        }

        @Override
        public KeyedStateStore globalState() {
            throw new UnsupportedOperationException("keyed global state in a GPU window function");
        }

        @Override
        public <X> void output(OutputTag<X> outputTag, X value) {
            output.collect(outputTag, new StreamRecord<>(value, window.maxTimestamp()));
        }
    }

    /** The key of a fired row: the Long itself, or the dictionary's key for an id. */
    private Object key(long id) { return dict == null ? (Object) id : dict.keyOf(id); }

    private void emitLate() {
        int got;
        while ((got = nativeDrainLate(handle, lKey, lTs, lVal, batchCapacity)) > 0) {
            for (int i = 0; i < got; i++) {
                Object v = doubleValue != null ? (Object) lVal.getDouble(i * 8) : lVal.getLong(i * 8);
                output.collect(lateDataTag, new StreamRecord<>(Tuple2.of(key(lKey.getLong(i * 8)), v), lTs.getLong(i * 8)));
            }
            if (got < batchCapacity) break;
        }
    }

    @Override
    public void processWatermark(Watermark mark) throws Exception {
        if (handleDeferred) {  // staggered, no element yet: nothing can fire; remember the watermark
            deferredWatermark = Math.max(deferredWatermark, mark.getTimestamp());
            super.processWatermark(mark);
            return;
        }
        flush();
        currentWm = mark.getTimestamp();
        nativeAdvanceWatermark(handle, mark.getTimestamp());
        emitRows();
        if (wide()) releaseElements(mark.getTimestamp());
        super.processWatermark(mark);  // forward after the fired rows
    }

    /** A batch's elements leave the log once every window they could fall in is cleaned up
     *  (maxTs + size - 1 + allowed lateness <= watermark: WindowOperator.cleanupTime), the rule
     *  the native payload log releases by. */
    private void releaseElements(long wm) {
        while (!batches.isEmpty()) {
            long[] b = batches.peekFirst();
            long ct = b[1] + (size - 1);
            ct = ct < b[1] ? Long.MAX_VALUE : ct;  // saturate like the window's cleanup time
            ct = ct + lateness < ct ? Long.MAX_VALUE : ct + lateness;
            if (b[1] != Long.MIN_VALUE && ct > wm) break;
            elements.releaseUpTo(b[0]);
            batches.pollFirst();
        }
    }

    /** Non-Long keys <-> dense int64 ids (the GPU keys), with each key's hashCode.  Ids are never
     *  released: the dictionary holds every key the subtask has seen (one HashMap entry and one
     *  list slot per distinct key) for the operator's lifetime, like the reference's heap backend
     *  holds the key objects of live state, but also for keys whose windows are all cleaned; a job
     *  with an unbounded key space (session ids) should key by a Long, which needs no dictionary. */
    static final class KeyDictionary<T> {
        private final HashMap<T, Long> ids = new HashMap<>();
        private final ArrayList<T> keys = new ArrayList<>();

        long idOf(T key) {
            Long id = ids.get(key);
            if (id == null) {
                id = (long) keys.size();
                ids.put(key, id);
                keys.add(key);
            }
            return id;
        }

        T keyOf(long id) { return keys.get((int) id); }
    }

    /** Elements by arrival sequence, a growable ring: append at the end, release from the start. */
    private static final class ElementLog<T> {
        private Object[] ring = new Object[1024];
        private long start, end;

        long append(T v) {
            if (end - start == ring.length) {
                Object[] r = new Object[ring.length * 2];
                for (long q = start; q < end; q++) r[(int) (q % r.length)] = ring[(int) (q % ring.length)];
                ring = r;
            }
            ring[(int) (end % ring.length)] = v;
            return end++;
        }

        @SuppressWarnings("unchecked")
        T get(long seq) {
            if (seq < start || seq >= end) throw new IllegalStateException("element " + seq + " was released");
            return (T) ring[(int) (seq % ring.length)];
        }

        long end() { return end; }

        void releaseUpTo(long seqEnd) {
            for (; start < seqEnd; start++) ring[(int) (start % ring.length)] = null;
        }
    }

    @Override
    public void endInput() throws Exception { processWatermark(Watermark.MAX_WATERMARK); }

    @Override
    public void close() throws Exception {
        if (windowFunction != null) FunctionUtils.closeFunction(windowFunction);
        if (handle != 0) nativeDestroy(handle);
        handle = 0;
        super.close();
    }

    public long numLateRecordsDropped() { return nativeLateDropped(handle); }

    private static native int nativeStageAlloc(long h, int slots, int cap);
    private static native ByteBuffer nativeStageColumn(long h, int slot, int which, int cap);
    private static native void nativeIngestStage(long h, int slot, int n, int cols);
    /** gw_stage_send: a complete slot over PCIe ahead of its nativeIngestStage (up to two batches ahead). */
    private static native void nativeStageSend(long h, int slot, int n, int cols);
    private static native long nativeStaggerOffset(int stagger, long processingTime, double random01, long size,
                                                   long globalOffset);
    private static native long nativeCreate(int assigner, int trigger, long size, long slide, long offset, long gap,
                                            long lateness, int agg, int maxParallelism, int parallelism,
                                            int subtask, int device, int flags, long capacityHint, long maxBatch);
    private static native void nativeIngest(long h, int n, ByteBuffer keys, ByteBuffer keyHashes, ByteBuffer ts,
                                            ByteBuffer values);
    private static native long nativeAdvanceWatermark(long h, long wm);
    private static native int nativeDrain(long h, ByteBuffer key, ByteBuffer start, ByteBuffer end, ByteBuffer result,
                                          int cap);
    private static native void nativeIngestPayload(long h, int n, ByteBuffer keys, ByteBuffer keyHashes, ByteBuffer ts,
                                                   ByteBuffer values, ByteBuffer payload);
    private static native int nativeDrainPayload(long h, ByteBuffer key, ByteBuffer start, ByteBuffer end,
                                                 ByteBuffer result, ByteBuffer payload, int cap);
    private static native long nativeLateDropped(long h);
    private static native void nativeDestroy(long h);
    private static native void nativeFlush(long h);
    private static native byte[] nativeSnapshot(long h, int kgLo, int kgHi);
    private static native byte[] nativeSliceKeyGroup(byte[] blob, int kg);
    private static native void nativeRestore(long h, byte[] blob);
    private static native long[] nativeSnapshotKeys(byte[] blob);
    private static native void nativeRemapKeys(byte[] blob, long[] from, long[] to);
    private static native long[] nativeSnapshotPayloads(byte[] blob, long[] maxEnd);
    private static native void nativeRemapPayloads(byte[] blob, long[] from, long[] to);
    private static native int nativeDrainLate(long h, ByteBuffer key, ByteBuffer ts, ByteBuffer value, int cap);
    /** The keyBy exchange's receive columns (GpuKeyByExchange.batch, produced on `stream`)
     *  straight into the operator. */
    static native void nativeIngestDevice(long h, long n, long keyPtr, long hashPtr, long tsPtr, long valuePtr,
                                          long stream);
}
