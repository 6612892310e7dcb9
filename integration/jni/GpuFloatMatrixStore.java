package com.intel.distml.util.store;

import com.intel.distml.util.DataDesc;
import com.intel.distml.util.KeyCollection;

import java.io.DataInputStream;
import java.io.DataOutputStream;
import java.io.IOException;

/**
 * FloatMatrixStore whose shard lives in HBM (GpuDataStore, libdistml_ps): every method the
 * parent implements on localData runs on the GPU, so the JVM heap holds no copy of
 * the shard (FloatMatrixStore.java:28-37, Iter :241-269). localData stays null until snapshot()
 * fills it from the device — iter() does, so callers that downcast to FloatMatrixStore and iterate read the trained values.
 * Created by GpuStores.createStore (the DataStore.createStore dispatch, DataStore.java:50-92).
 */
public class GpuFloatMatrixStore extends FloatMatrixStore {
    private final DataDesc format;
    private final int device;
    private GpuDataStore gpu;

    public GpuFloatMatrixStore(DataDesc format, int device) {
        this.format = format;
        this.device = device;
    }

    /** FloatMatrixStore.init without the heap arrays: the shard is zero-filled in HBM. */
    public void init(KeyCollection keys, int cols) {
        gpu = new GpuDataStore(format, GpuStores.range(keys), cols, device);
        localRows = keys;
        rowSize = cols;
    }

    public KeyCollection rows() { return localRows; }
    public int rowSize() { return rowSize; }
    public byte[] handleFetch(DataDesc format, KeyCollection rows) { return gpu.handleFetch(format, rows); }
    public void writeAll(DataOutputStream os) throws IOException { gpu.writeAll(os); }
    public void readAll(DataInputStream is) throws IOException { gpu.readAll(is); }
    public void syncTo(DataOutputStream os, int fromRow, int toRow) throws IOException { gpu.syncTo(os, fromRow, toRow); }
    public void syncFrom(DataInputStream is, int fromRow, int toRow) throws IOException { gpu.syncFrom(is, fromRow, toRow); }
    /** The device store behind this one (pinned wire ingest, handlePushDirect). */
    public GpuDataStore gpu() { return gpu; }
    public void close() { gpu.close(); }
    public void handlePush(DataDesc format, byte[] data) { gpu.handlePush(format, data); }
    /** Unseeded in the reference (FloatMatrixStore.java:39-51): same distribution. */
    public void rand() { gpu.rand(); }
    public void set(String value) { gpu.set(value); }
    /** FloatMatrixStore.zero(String) = setValue(0f) (:57-59). */
    public void zero(String value) { gpu.fill(0f); }

    /** Fill the parent's localData from the device shard (every accepted
     *  push applied): the state the reference store holds at this point. */
    public void snapshot() {
        if (localData == null) localData = new float[(int) localRows.size()][rowSize];
        gpu.snapshot(0, DataDesc.ELEMENT_TYPE_FLOAT, localData);
    }

    /** FloatMatrixStore.Iter over a snapshot taken now. */
    public Iter iter() {
        snapshot();
        return super.iter();
    }
}
