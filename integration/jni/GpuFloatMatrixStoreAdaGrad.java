package com.intel.distml.util.store;

import com.intel.distml.util.DataDesc;
import com.intel.distml.util.KeyCollection;

import java.io.DataInputStream;
import java.io.DataOutputStream;
import java.io.IOException;

/**
 * FloatMatrixStoreAdaGrad whose shard lives in HBM (GpuDataStore, libdistml_ps): every method the
 * parent implements on localData runs on the GPU, so the JVM heap holds no copy of
 * the shard (FloatMatrixStoreAdaGrad.java:38-53, Iter :308-337). localData stays null until snapshot()
 * fills it from the device — iter() does, so callers that downcast to FloatMatrixStoreAdaGrad and iterate read the trained values.
 * Created by GpuStores.createStore (the DataStore.createStore dispatch, DataStore.java:50-92).
 */
public class GpuFloatMatrixStoreAdaGrad extends FloatMatrixStoreAdaGrad {
    private final DataDesc format;
    private final int device;
    private GpuDataStore gpu;

    public GpuFloatMatrixStoreAdaGrad(DataDesc format, int device) {
        this.format = format;
        this.device = device;
    }

    /** FloatMatrixStoreAdaGrad.init without the heap arrays: the shard is zero-filled in HBM. */
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

    /** handlePush on the device, then the reference's per-push report of the largest
     *  delta (FloatMatrixStoreAdaGrad.java:246; maxDeltaRow is the (int) key, :273-277). */
    public void handlePush(DataDesc format, byte[] data) {
        gpu.handlePush(format, data);
        final int[] rc = new int[2];
        maxDelta = gpu.maxDelta(rc);
        maxDeltaRow = rc[0];
        maxDeltaCol = rc[1];
        System.out.println("max delta: " + maxDeltaRow + ", " + maxDeltaCol + ", " + maxDelta);
    }
    /** Unseeded in the reference (FloatMatrixStore.java:39-51): same distribution. */
    public void rand() { gpu.rand(); }
    public void set(String value) { gpu.set(value); }
    /** FloatMatrixStore.zero(String) = setValue(0f) (:57-59). */
    public void zero(String value) { gpu.fill(0f); }
    /** setAlphaValue(initialAlpha) on the device, then the three fields (:77-82). */
    public void setAlpha(float initialAlpha, float minAlpha, float factor) {
        gpu.setAlpha(initialAlpha, minAlpha, factor);
        this.initialAlpha = initialAlpha;
        this.minAlpha = minAlpha;
        this.factor = factor;
    }

    /** Fill the parent's localData / alpha / delta from the device shard (every accepted
     *  push applied): the state the reference store holds at this point. */
    public void snapshot() {
        if (localData == null) localData = new float[(int) localRows.size()][rowSize];
        gpu.snapshot(0, DataDesc.ELEMENT_TYPE_FLOAT, localData);
        if (alpha == null) alpha = new float[(int) localRows.size()][rowSize];
        if (delta == null) delta = new float[(int) localRows.size()][rowSize];
        gpu.snapshot(1, DataDesc.ELEMENT_TYPE_FLOAT, alpha);
        gpu.snapshot(2, DataDesc.ELEMENT_TYPE_FLOAT, delta);
    }

    /** FloatMatrixStoreAdaGrad.Iter over a snapshot taken now. */
    public Iter iter() {
        snapshot();
        return super.iter();
    }
}
