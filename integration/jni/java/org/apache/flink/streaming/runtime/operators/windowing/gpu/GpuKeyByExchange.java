package org.apache.flink.streaming.runtime.operators.windowing.gpu;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;

/**
 * The keyBy shuffle of a GPU window job through libgpuwin's RCCL communicator
 * (include/gpuwin.h gw_exchange_*): replaces KeyGroupStreamPartitioner.selectChannel
 * (KeyGroupStreamPartitioner.java:55-64) + RecordWriter + the Netty transport for the
 * columns of one watermark batch, and StatusWatermarkValve's minimum over channels.
 * One instance per subtask / GPU; every subtask calls {@link #batch} once per batch.
 * Subtask 0 creates the communicator id ({@link #uniqueId}); the job ships it to the
 * others (e.g. through the operator coordinator) before {@link #open}.
 */
public final class GpuKeyByExchange implements AutoCloseable {
    public static final int ID_BYTES = 128;

    private long handle;
    private final ByteBuffer out = ByteBuffer.allocateDirect(7 * 8).order(ByteOrder.nativeOrder());

    public static byte[] uniqueId() {
        ByteBuffer id = ByteBuffer.allocateDirect(ID_BYTES);
        nativeUniqueId(id);
        byte[] b = new byte[ID_BYTES];
        id.get(b);
        return b;
    }

    public GpuKeyByExchange open(int parallelism, int subtask, byte[] id, int device, int maxParallelism) {
        ByteBuffer b = ByteBuffer.allocateDirect(ID_BYTES);
        b.put(id).flip();
        handle = nativeCreate(parallelism, subtask, b, device, maxParallelism);
        return this;
    }

    /** One watermark batch: device columns in (addresses; 0 = absent) and the watermark the
     *  source emitted after them.  Returns {n, key, keyHash, ts, value, minWatermark,
     *  ingestStream}: the records this subtask owns, in the exchange's receive columns (valid
     *  until the next-but-one call), the minimum watermark over the subtasks
     *  (StatusWatermarkValve, carried by the same all-to-all as the counts: one host wait per
     *  batch), and the stream to hand to GpuWindowOperator.nativeIngestDevice. */
    public long[] batch(long n, long keyPtr, long hashPtr, long tsPtr, long valuePtr, long watermark, long stream) {
        nativeBatch(handle, n, keyPtr, hashPtr, tsPtr, valuePtr, watermark, stream, out);
        long[] r = new long[7];
        for (int i = 0; i < 7; i++) r[i] = out.getLong(8 * i);
        return r;
    }

    /** {@link #batch} in two halves, so the host never waits between batches: begin batch
     *  b + 1 (partition + the count all-to-all, no wait), then finish batch b (its one bounded
     *  wait, the sends; returns what {@link #batch} returns).  At most two batches begun and not
     *  finished; both halves on one stream; every subtask begins and finishes in the same order. */
    public void begin(long n, long keyPtr, long hashPtr, long tsPtr, long valuePtr, long watermark, long stream) {
        nativeBegin(handle, n, keyPtr, hashPtr, tsPtr, valuePtr, watermark, stream);
    }

    public long[] finish(long stream) {
        nativeFinish(handle, stream, out);
        long[] r = new long[7];
        for (int i = 0; i < 7; i++) r[i] = out.getLong(8 * i);
        return r;
    }

    public long minWatermark(long wm, long stream) { return nativeMinWatermark(handle, wm, stream); }

    /** Bound of every host wait of the exchange (include/gpuwin.h gw_exchange_set_timeout;
     *  default 60 s, 0: none).  A dead or diverging peer, an asynchronous RCCL error or a
     *  stream error aborts the communicator: {@link #batch} / {@link #minWatermark} then throw
     *  IllegalStateException (the task fails and restarts from its checkpoint, as a failed
     *  network channel fails it in the reference), and so does every later call. */
    public void setTimeout(long timeoutMs) { nativeSetTimeout(handle, timeoutMs); }

    /** From the next batch on, records whose key fits 32 bits, value 28 bits and pane the 16
     *  after the watermark's travel as 8-byte words (include/gpuwin.h gw_exchange_enable_packing):
     *  for a tumbling / sliding operator with size >= slide, no late side output and an integer
     *  aggregate.  Every subtask must call it alike. */
    public void enablePacking(long size, long slide, long offset, boolean withValues) {
        nativeEnablePacking(handle, size, slide, offset, withValues);
    }

    @Override
    public void close() {
        if (handle != 0) nativeDestroy(handle);
        handle = 0;
    }

    private static native void nativeUniqueId(ByteBuffer id);
    private static native long nativeCreate(int nranks, int rank, ByteBuffer id, int device, int maxParallelism);
    private static native void nativeDestroy(long h);
    private static native void nativeBatch(long h, long n, long keyPtr, long hashPtr, long tsPtr, long valuePtr,
                                           long watermark, long stream, ByteBuffer out);
    private static native long nativeMinWatermark(long h, long wm, long stream);
    private static native void nativeEnablePacking(long h, long size, long slide, long offset, boolean withValues);
    private static native void nativeSetTimeout(long h, long timeoutMs);
    private static native void nativeBegin(long h, long n, long keyPtr, long hashPtr, long tsPtr, long valuePtr,
                                           long watermark, long stream);
    private static native void nativeFinish(long h, long stream, ByteBuffer out);
}
