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
 * DataStore backed by libdistml_ps (MI355X, HBM-resident shard, HIP kernels).
 * Drop-in for the seven typed stores that DataStore.createStore returns
 * (DataStore.java:50-92): same methods, same byte layouts, same exceptions.
 * Native methods are implemented in dml_jni.cc over include/distml_ps.h.
 */
public class GpuDataStore extends DataStore {
    static { System.loadLibrary("distml_jni"); }

    private final long handle;          // dml_store*
    private final KeyRange localRows;
    private final int rowSize;

    public GpuDataStore(DataDesc format, KeyRange keys, int cols, int device) {
        this.localRows = keys;
        this.rowSize = format.dataType == DataDesc.DATA_TYPE_MATRIX ? cols : 1;
        this.handle = nativeCreate(format.dataType, format.keyType, format.valueType,
                format.denseRow ? 1 : 0, format.denseColumn ? 1 : 0, format.adaGrad ? 1 : 0,
                keys.firstKey, keys.lastKey, cols, device, 0);
    }

    public KeyCollection rows() { return localRows; }
    public int rowSize() { return rowSize; }

    public void zero() { nativeFill(handle, 0.0); }
    public void set(String value) { nativeFill(handle, Float.parseFloat(value)); }
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
    public void syncTo(DataOutputStream os, int fromRow, int toRow) throws IOException {
        byte[] all = nativeWriteAll(handle);
        int rec = all.length / (int) localRows.size();
        os.write(all, fromRow * rec, (toRow - fromRow + 1) * rec);
    }
    public void syncFrom(DataInputStream is, int fromRow, int toRow) throws IOException {
        byte[] all = nativeWriteAll(handle);
        int rec = all.length / (int) localRows.size();
        is.readFully(all, fromRow * rec, (toRow - fromRow + 1) * rec);
        nativeReadAll(handle, all);
    }

    public void close() { nativeDestroy(handle); }

    private static native long nativeCreate(int dataType, int keyType, int valueType, int denseRow, int denseColumn,
                                            int adaGrad, long firstKey, long lastKey, int cols, int device, int flags);
    private static native void nativePush(long h, byte[] data);
    private static native byte[] nativeFetch(long h, long[] keys);
    private static native byte[] nativeFetchRange(long h, long first, long last);
    private static native byte[] nativeWriteAll(long h);
    private static native void nativeReadAll(long h, byte[] be);
    private static native long nativeShardBytes(long h);
    private static native void nativeFill(long h, double v);
    private static native void nativeSetAlpha(long h, float a, float min, float factor);
    private static native void nativeDestroy(long h);
}
