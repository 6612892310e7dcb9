package com.intel.distml.util.store;

import com.intel.distml.util.DataDesc;
import com.intel.distml.util.DataStore;
import com.intel.distml.util.KeyCollection;
import com.intel.distml.util.KeyRange;

import java.io.DataInputStream;
import java.io.DataOutputStream;
import java.io.IOException;
import java.util.Iterator;

/**
 * DataStore backed by libdistml_ps (MI355X, HBM-resident shard, HIP kernels): the
 * push / fetch / checkpoint / init methods of the seven typed stores that
 * DataStore.createStore returns (DataStore.java:50-92), same byte layouts, same
 * exceptions. Callers that downcast a store to its concrete class and iterate it
 * (LogisticRegression.scala:290-291, Word2Vec.scala:814-817) get the typed
 * subclasses from GpuStores.createStore (GpuDoubleArrayStore extends
 * DoubleArrayStore, ...), which delegate here and fill the parent's localData
 * from a snapshot of the shard in iter().
 * Native methods are implemented in dml_jni.cc over include/distml_ps.h.
 */
public class GpuDataStore extends DataStore {
    static { System.loadLibrary("distml_jni"); }

    private final long handle;          // dml_store*
    private final KeyRange localRows;
    private final int rowSize;
    private final int valueBytes;
    private final boolean floatMatrix;  // FloatMatrixStore / FloatMatrixStoreAdaGrad: the stores set() acts on

    public GpuDataStore(DataDesc format, KeyRange keys, int cols, int device) {
        this.localRows = keys;
        this.rowSize = format.dataType == DataDesc.DATA_TYPE_MATRIX ? cols : 1;
        this.valueBytes = format.valueType == DataDesc.ELEMENT_TYPE_DOUBLE ? 8 : 4;
        this.floatMatrix = format.dataType == DataDesc.DATA_TYPE_MATRIX
                && format.valueType == DataDesc.ELEMENT_TYPE_FLOAT;
        this.handle = nativeCreate(format.dataType, format.keyType, format.valueType,
                format.denseRow ? 1 : 0, format.denseColumn ? 1 : 0, format.adaGrad ? 1 : 0,
                keys.firstKey, keys.lastKey, cols, device, 0);
    }

    public KeyCollection rows() { return localRows; }
    public int rowSize() { return rowSize; }

    /** DataStore.rand() / PSActor OP_RAND (PSActor.java:181-201): DoubleMatrixStore's
     *  Random(1L) unit-norm |gaussian| rows, value for value (DoubleMatrixStore.java:192-207);
     *  FloatMatrixStore's (nextInt(100)/100f - 0.5f)/rowSize from an unseeded generator
     *  (FloatMatrixStore.java:39-51); a no-op for the others. */
    public void rand() { nativeRand(handle, System.nanoTime()); }
    /** DataStore.zero() is a no-op on every store (DataStore.java:24): the float stores'
     *  zero(String) is an overload, so OP_ZERO (PSActor.java:185-188) changes nothing. */
    public void zero() { }
    /** set(String) fills only the float matrix stores (FloatMatrixStore.java:53-55,
     *  FloatMatrixStoreAdaGrad.java:69-71); DataStore's default is a no-op (DataStore.java:26). */
    public void set(String value) {
        if (floatMatrix) nativeFill(handle, Float.parseFloat(value));
    }
    /** FloatMatrixStore.setValue (FloatMatrixStore.java:61-71): zero(String) fills 0f. */
    void fill(float v) { nativeFill(handle, v); }
    public void setAlpha(float initialAlpha, float minAlpha, float factor) {
        nativeSetAlpha(handle, initialAlpha, minAlpha, factor);
    }

    /** PSAgent.handle calls this under synchronized(store) (PSAgent.java:278-280). */
    public void handlePush(DataDesc format, byte[] data) { nativePush(handle, data); }

    public byte[] handleFetch(DataDesc format, KeyCollection rows) {
        KeyCollection keys = localRows.intersect(rows);
        if (keys instanceof KeyRange) {
            KeyRange r = (KeyRange) keys;
            return nativeFetchRange(handle, r.firstKey, r.lastKey);
        }
        long[] ks = new long[(int) keys.size()];
        int i = 0;
        for (Iterator<Long> it = keys.iterator(); it.hasNext(); ) ks[i++] = it.next();
        return nativeFetch(handle, ks);
    }

    public void writeAll(DataOutputStream os) throws IOException { os.write(nativeWriteAll(handle)); }
    public void readAll(DataInputStream is) throws IOException {
        byte[] b = new byte[(int) nativeShardBytes(handle)];
        is.readFully(b);
        nativeReadAll(handle, b);
    }
    /** PSSync.java:131 — rows fromRow..toRow, big-endian, moved by the device. */
    public void syncTo(DataOutputStream os, int fromRow, int toRow) throws IOException {
        os.write(nativeSyncTo(handle, fromRow, toRow));
    }
    /** PSSync.java:160 — intended row layout (the reference's matrix syncFrom shadows rowSize). */
    public void syncFrom(DataInputStream is, int fromRow, int toRow) throws IOException {
        int last = Math.min(toRow, (int) localRows.size() - 1);
        byte[] b = new byte[Math.max(0, last - fromRow + 1) * rowSize * valueBytes];
        is.readFully(b);
        nativeSyncFrom(handle, fromRow, toRow, b);
    }

    /** Wire ingest: a pinned DirectByteBuffer the NIO channel reads PushRequests into. */
    public static java.nio.ByteBuffer allocatePinned(long bytes) { return nativeHostAlloc(bytes); }
    public static void freePinned(java.nio.ByteBuffer b) { nativeHostFree(b); }
    /** handlePush of the record bytes at buf[offset, offset + len) (no JVM heap copy). */
    public void handlePushDirect(java.nio.ByteBuffer buf, int offset, int len) {
        nativePushDirect(handle, buf, offset, len);
    }

    public void close() { nativeDestroy(handle); }

    /** Copy the shard (which 0), or AdaGrad's alpha (1) / delta (2), into dst: a
     *  T[rows][rowSize] for matrices, a T[rows] for arrays; T = the element type
     *  DataDesc names (ELEMENT_TYPE_INT / FLOAT / DOUBLE). Every accepted push is
     *  applied first (dml_store_read_rows). */
    void snapshot(int which, int elemType, Object dst) {
        nativeSnapshot(handle, which, elemType, dst instanceof Object[] ? 2 : 1, dst);
    }
    /** FloatMatrixStoreAdaGrad's maxDelta; rowCol receives maxDeltaRow, maxDeltaCol. */
    float maxDelta(int[] rowCol) { return nativeMaxDelta(handle, rowCol); }

    static native long nativeCreate(int dataType, int keyType, int valueType, int denseRow, int denseColumn,
                                            int adaGrad, long firstKey, long lastKey, int cols, int device, int flags);
    static native void nativePush(long h, byte[] data);
    static native byte[] nativeFetch(long h, long[] keys);
    static native byte[] nativeFetchRange(long h, long first, long last);
    static native byte[] nativeWriteAll(long h);
    static native void nativeReadAll(long h, byte[] be);
    static native long nativeShardBytes(long h);
    static native byte[] nativeSyncTo(long h, int from, int to);
    static native void nativeSyncFrom(long h, int from, int to, byte[] be);
    static native java.nio.ByteBuffer nativeHostAlloc(long bytes);
    static native void nativeHostFree(java.nio.ByteBuffer b);
    static native void nativePushDirect(long h, java.nio.ByteBuffer b, int offset, int len);
    static native void nativeFill(long h, double v);
    static native void nativeRand(long h, long seed);
    static native void nativeSetAlpha(long h, float a, float min, float factor);
    static native void nativeDestroy(long h);
    static native void nativeSnapshot(long h, int which, int elemType, int dims, Object dst);
    static native float nativeMaxDelta(long h, int[] rowCol);
}
