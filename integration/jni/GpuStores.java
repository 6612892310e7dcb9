package com.intel.distml.util.store;

import com.intel.distml.util.DataDesc;
import com.intel.distml.api.DMatrix;
import com.intel.distml.util.DataStore;
import com.intel.distml.util.KeyCollection;
import com.intel.distml.util.KeyRange;

/**
 * DataStore.createStore (DataStore.java:50-92) for GPU stores: the same dispatch on
 * the matrix's DataDesc, returning the typed subclass of the store the reference
 * would create (GpuDoubleArrayStore for a DoubleArrayStore, ...), so that code which
 * downcasts and iterates (LogisticRegression.scala:290-291, Word2Vec.scala:814-817)
 * works unchanged. Route DataStore.createStore here (INTEGRATION.md).
 */
public final class GpuStores {
    private GpuStores() { }

    public static DataStore createStore(int serverIndex, DMatrix matrix, int device) {
        DataDesc format = matrix.getFormat();
        KeyCollection keys = matrix.partitions[serverIndex];
        int cols = (int) matrix.getColKeys().size();
        if (format.dataType == DataDesc.DATA_TYPE_ARRAY) {
            if (format.valueType == DataDesc.ELEMENT_TYPE_INT) {
                GpuIntArrayStore store = new GpuIntArrayStore(format, device);
                store.init(keys);
                return store;
            } else if (format.valueType == DataDesc.ELEMENT_TYPE_DOUBLE) {
                GpuDoubleArrayStore store = new GpuDoubleArrayStore(format, device);
                store.init(keys);
                return store;
            } else if (format.valueType == DataDesc.ELEMENT_TYPE_FLOAT) {
                GpuFloatArrayStore store = new GpuFloatArrayStore(format, device);
                store.init(keys);
                return store;
            }
        } else {
            if (format.valueType == DataDesc.ELEMENT_TYPE_INT) {
                GpuIntMatrixStore store = new GpuIntMatrixStore(format, device);
                store.init(keys, cols);
                return store;
            } else if (format.valueType == DataDesc.ELEMENT_TYPE_DOUBLE) {
                GpuDoubleMatrixStore store = new GpuDoubleMatrixStore(format, device);
                store.init(keys, cols);
                return store;
            } else if (format.valueType == DataDesc.ELEMENT_TYPE_FLOAT) {
                if (format.adaGrad) {
                    GpuFloatMatrixStoreAdaGrad store = new GpuFloatMatrixStoreAdaGrad(format, device);
                    store.init(keys, cols);
                    return store;
                }
                GpuFloatMatrixStore store = new GpuFloatMatrixStore(format, device);
                store.init(keys, cols);
                return store;
            }
        }
        throw new IllegalArgumentException("Unrecognized matrix type: " + matrix.getClass().getName());
    }

    /** The GPU stores take KeyRange shards (KeyRange.linearSplit, KeyRange.java:68-80);
     *  a KeyHash shard aliases keys (SURVEY defect 2) and is refused. */
    static KeyRange range(KeyCollection keys) {
        if (!(keys instanceof KeyRange))
            throw new RuntimeException("Only KeyRange is allowed in GPU server storage");
        return (KeyRange) keys;
    }
}
