package com.intel.distml.util.store;

import com.intel.distml.util.DataDesc;

/**
 * One PS process per GPU: shard `rank` of KeyRange.linearSplit(world)
 * (KeyRange.java:68-80) as an HBM-resident store, with device-resident
 * full-range pushes pre-reduced in push order, reduce-scattered over xGMI
 * (RCCL) and applied by their owner — include/distml_ps.h dml_group_*.
 * Rank 0 calls uniqueId() and the PS control plane (PSActor messages) hands the
 * 128 bytes to every rank before they construct their group.
 */
public class GpuShardGroup implements AutoCloseable {
    static { System.loadLibrary("distml_jni"); }

    private long handle;  // dml_group*

    public static byte[] uniqueId() { return nativeUniqueId(); }

    public GpuShardGroup(byte[] uniqueId, int world, int rank, int device, DataDesc format,
                         long totalRows, int cols, int pieces) {
        handle = nativeGroupCreate(uniqueId, world, rank, device, format.dataType, format.keyType,
                format.valueType, format.denseRow ? 1 : 0, format.denseColumn ? 1 : 0,
                format.adaGrad ? 1 : 0, totalRows, cols, pieces);
    }

    /** Device pointers (HBM, this GPU) and byte lengths of up to 64 full-range pushes. */
    public void pushFullRange(long[] devPtrs, long[] lens) { nativeGroupPush(handle, devPtrs, lens, 0); }

    /**
     * Exact path for AdaGrad, int32-checked, array or key-subset pushes: split by owner
     * (SparseMatrix.push's per-partition split), exchanged with RCCL send/recv, applied by
     * each owner in rank-major push order. Every rank passes the same number of pushes.
     */
    public void pushExchange(long[] devPtrs, long[] lens) { nativeGroupPush(handle, devPtrs, lens, 1); }

    /** AdaGrad with many pushes per rank: Σu and Σu² reduce-scattered, within 1e-6 (not bit-exact). */
    public void pushMoments(long[] devPtrs, long[] lens) { nativeGroupPush(handle, devPtrs, lens, 2); }

    /**
     * Pushes the client already split to this shard (SparseMatrix.java:46-60): the exact
     * ordered apply, after every earlier call of this group. Push to storeHandle() directly
     * only after flush(): the group applies its calls in call order.
     */
    public void pushLocal(long[] devPtrs, long[] lens) { nativeGroupPush(handle, devPtrs, lens, 3); }

    /** Every call applied; throws the first deferred key / repeated-row error. */
    public void flush() { nativeGroupFlush(handle); }

    /** dml_store* of this rank's shard (owned by the group), for fetch / checkpoint after flush(). */
    public long storeHandle() { return nativeGroupStore(handle); }

    public void close() {
        if (handle != 0) {
            nativeGroupDestroy(handle);
            handle = 0;
        }
    }

    private static native byte[] nativeUniqueId();
    private static native long nativeGroupCreate(byte[] id, int world, int rank, int device, int dataType,
                                                 int keyType, int valueType, int denseRow, int denseColumn,
                                                 int adaGrad, long totalRows, int cols, int pieces);
    private static native void nativeGroupPush(long g, long[] devPtrs, long[] lens, int mode);
    private static native void nativeGroupFlush(long g);
    private static native long nativeGroupStore(long g);
    private static native void nativeGroupDestroy(long g);
}
