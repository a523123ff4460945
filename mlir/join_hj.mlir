// join_hj.mlir -- the reference's @main (join_v2.mlir:607-730) with the GPU
// join replaced by libhj.so's memref ABI (include/hj.h).  The relations and
// the final check still come from the reference's shared_stuff/shared.cpp
// (initRelationR/S, check, startTimer/endTimer), so this module is a literal
// drop-in: same inputs, same check, same stdout protocol (result size, then
// 1/0/-1).  Run with mlir/run_hj.sh (needs an MLIR toolchain; none is in the
// build container -- see INTEGRATION.md).
module {
    memref.global constant @buildRelationRows : memref<1xindex> = dense<[1024]>
    memref.global constant @probeRelationRows : memref<1xindex> = dense<[1024]>

    func.func private @initRelationR(memref<?xi32>)
    func.func private @initRelationS(memref<?xi32>)
    func.func private @check(memref<?xi32>, memref<?xi32>, memref<?xi32>, memref<?xi32>) -> i32
    func.func private @printMemrefI32(memref<*xi32>)
    func.func private @startTimer()
    func.func private @endTimer()

    // libhj.so: two-phase form mirroring @countRows / @probeRelation
    func.func private @hj_count_i32(memref<?xi32>, memref<?xi32>) -> i64
    func.func private @hj_probe_i32(memref<?xi32>, memref<?xi32>, memref<?xi32>, memref<?xi32>) -> i32
    // libhj.so: two-memref-in / one-memref-out form (C interface)
    func.func private @hj_join_i32(memref<?xi32>, memref<?xi32>) -> memref<?x2xi32>
        attributes {llvm.emit_c_interface}

    func.func @debugI32(%v: i32) {
        %m = memref.alloc() : memref<i32>
        memref.store %v, %m[] : memref<i32>
        %c = memref.cast %m : memref<i32> to memref<*xi32>
        func.call @printMemrefI32(%c) : (memref<*xi32>) -> ()
        memref.dealloc %m : memref<i32>
        return
    }

    func.func @main() {
        %c0 = arith.constant 0 : index
        %c1 = arith.constant 1 : index
        %nRm = memref.get_global @buildRelationRows : memref<1xindex>
        %nR = memref.load %nRm[%c0] : memref<1xindex>
        %nSm = memref.get_global @probeRelationRows : memref<1xindex>
        %nS = memref.load %nSm[%c0] : memref<1xindex>

        %R = memref.alloc(%nR) : memref<?xi32>
        func.call @initRelationR(%R) : (memref<?xi32>) -> ()
        %S = memref.alloc(%nS) : memref<?xi32>
        func.call @initRelationS(%S) : (memref<?xi32>) -> ()

        // count -> allocate -> probe (join_v2.mlir:672-696)
        func.call @startTimer() : () -> ()
        %m64 = func.call @hj_count_i32(%R, %S) : (memref<?xi32>, memref<?xi32>) -> i64
        func.call @endTimer() : () -> ()
        %m32 = arith.trunci %m64 : i64 to i32
        func.call @debugI32(%m32) : (i32) -> ()
        %m = arith.index_cast %m64 : i64 to index
        %oR = memref.alloc(%m) : memref<?xi32>
        %oS = memref.alloc(%m) : memref<?xi32>
        func.call @startTimer() : () -> ()
        %rc = func.call @hj_probe_i32(%R, %S, %oR, %oS)
            : (memref<?xi32>, memref<?xi32>, memref<?xi32>, memref<?xi32>) -> i32
        func.call @endTimer() : () -> ()
        %ok = func.call @check(%R, %S, %oR, %oS)
            : (memref<?xi32>, memref<?xi32>, memref<?xi32>, memref<?xi32>) -> i32
        func.call @debugI32(%ok) : (i32) -> ()

        // the one-memref-out form: result rows are (rowR, rowS)
        %pairs = func.call @hj_join_i32(%R, %S) : (memref<?xi32>, memref<?xi32>) -> memref<?x2xi32>
        %rows = memref.dim %pairs, %c0 : memref<?x2xi32>
        %rows32 = arith.index_cast %rows : index to i32
        func.call @debugI32(%rows32) : (i32) -> ()
        memref.dealloc %pairs : memref<?x2xi32>

        memref.dealloc %oR : memref<?xi32>
        memref.dealloc %oS : memref<?xi32>
        memref.dealloc %R : memref<?xi32>
        memref.dealloc %S : memref<?xi32>
        return
    }
}
