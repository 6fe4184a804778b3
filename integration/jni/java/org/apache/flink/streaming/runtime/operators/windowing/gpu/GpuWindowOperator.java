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
import java.util.HashMap;
import java.util.List;
import java.util.Map;

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
    public enum OutputMode { POSITIONAL, MIN_MAX_BY, AGGREGATE, KEYED_WINDOW }

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
        int subtask = getRuntimeContext().getTaskInfo().getIndexOfThisSubtask();
        int parallelism = getRuntimeContext().getTaskInfo().getNumberOfParallelSubtasks();
        int maxP = getRuntimeContext().getTaskInfo().getMaxNumberOfParallelSubtasks();
        int device = gpuIndex();
        final int flags = (lateDataTag != null ? 64 /* GW_FLAG_LATE_SIDE_OUTPUT */ : 0)
                | (mode == OutputMode.MIN_MAX_BY ? 512 /* GW_FLAG_BY_FIELD */ | (byFirst ? 0 : 1024 /* GW_FLAG_BY_LAST */)
                        : wide() ? 128 /* GW_FLAG_FIRST_ELEMENT */ : 0)
                | (parallelism > 1 ? 4 /* GW_FLAG_CHECK_KEY_GROUPS: a foreign key fails the batch */ : 0);
        handle = nativeCreate(assigner, trigger, size, slide, offset, gap, lateness, agg, maxP, parallelism,
                              subtask, device, flags, 1L << 24, batchCapacity);
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
        if (restored != null) {  // initializeState runs before open (StreamOperator.java:139)
            for (int i = 0; i < restored.size(); i++) {
                byte[] blob = restored.get(i);
                Map<Long, K> table = restoredKeys.get(i);
                if (table != null) {  // the blob's key ids -> this subtask's dictionary ids
                    long[] from = nativeSnapshotKeys(blob);
                    long[] to = new long[from.length];
                    for (int j = 0; j < from.length; j++) to[j] = dictionary().idOf(table.get(from[j]));
                    nativeRemapKeys(blob, from, to);
                }
                Map<Long, IN> firsts = restoredElements.get(i);
                if (firsts != null) {  // the first elements join this subtask's ElementLog
                    long[] maxEnd = new long[1];
                    long[] from = nativeSnapshotPayloads(blob, maxEnd);
                    long[] to = new long[from.length];
                    for (int j = 0; j < from.length; j++) to[j] = elements.append(firsts.get(from[j]));
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
                    default: row = Tuple4.of(key, oStart.getLong(i * 8), end, res);
                }
                // count windows: GlobalWindow.maxTimestamp() = Long.MAX_VALUE
                long tsOut = assigner == GW_COUNT_TUMBLING || assigner == GW_COUNT_SLIDING ? Long.MAX_VALUE : end - 1;
                output.collect(new StreamRecord<>(row, tsOut));
            }
            if (got < batchCapacity) break;
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
        flush();
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

    /** Non-Long keys <-> dense int64 ids (the GPU keys), with each key's hashCode. */
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
        if (handle != 0) nativeDestroy(handle);
        handle = 0;
        super.close();
    }

    public long numLateRecordsDropped() { return nativeLateDropped(handle); }

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
