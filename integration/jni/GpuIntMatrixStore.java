package com.intel.distml.util.store;

import com.intel.distml.util.DataDesc;
import com.intel.distml.util.KeyCollection;

import java.io.DataInputStream;
import java.io.DataOutputStream;
import java.io.IOException;

/**
 * IntMatrixStore whose shard lives in HBM (GpuDataStore, libdistml_ps): every method the
 * parent implements on localData runs on the GPU, so the JVM heap holds no copy of
 * the shard (IntMatrixStore.java:30-40). localData stays null until snapshot()
 * fills it from the device.
 * Created by GpuStores.createStore (the DataStore.createStore dispatch, DataStore.java:50-92).
 */
public class GpuIntMatrixStore extends IntMatrixStore {
    private final DataDesc format;
    private final int device;
    private GpuDataStore gpu;

    public GpuIntMatrixStore(DataDesc format, int device) {
        this.format = format;
        this.device = device;
    }

    /** IntMatrixStore.init without the heap arrays: the shard is zero-filled in HBM. */
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

    /** Fill the parent's localData from the device shard (every accepted
     *  push applied): the state the reference store holds at this point. */
    public void snapshot() {
        if (localData == null) localData = new int[(int) localRows.size()][rowSize];
        gpu.snapshot(0, DataDesc.ELEMENT_TYPE_INT, localData);
    }
}
