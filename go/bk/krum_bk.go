// Package main (drop-in file for DistributedML/Biscotti DistSys/).
//
// krum_bk.go replaces the go-python Multi-Krum call of DistSys/krum.go with the
// MI355X engine libbk.so (include/bk.h).  It keeps the verifier call surface:
//
//	func (krumval *KRUMValidator) initialize()                        krum.go:31-44
//	func (krumval *KRUMValidator) getTopKRUMIndex(deltas [][]float64) []int
//	                                                                  krum.go:100-166
//
// computeScores (krum.go:77-98), VerifyUpdateKRUM (:227-365),
// startKRUMDeadlineTimer (:178-224) and checkIfAccepted (:47-73) are unchanged.
// To adopt it: delete getTopKRUMIndex/initialize (and the pyKRUMFunc global)
// from krum.go, add this file, build with
//
//	CGO_CFLAGS="-I<repo>/include" CGO_LDFLAGS="-L<repo>/biscotti_amd -lbk -Wl,-rpath,<repo>/biscotti_amd" go build
//
// NOT BUILT IN THIS REPOSITORY: the build image has no Go toolchain (see
// INTEGRATION.md).  The C calls it makes are exercised from Python through the
// same ABI (tests/test_abi.py, tests/test_gpu_parity.py).
package main

/*
#cgo LDFLAGS: -lbk
#include <stdlib.h>
#include <string.h>
#include "bk.h"
*/
import "C"

import (
	"os"
	"runtime"
	"strconv"
	"unsafe"
)

var (
	bkCtx      *C.bk_ctx   // device 0's context (the group's rank 0 when bkGroup is set)
	bkGroup    *C.bk_group // BK_GPUS > 1: one process driving that many GPUs
	bkStage    unsafe.Pointer // C-owned pinned staging (cgo may not keep Go pointers)
	bkStageLen int64
)

// initialize binds the engine instead of pyKRUMFunc (krum.go:31-44).  With
// BK_GPUS=G (G > 1) the verifier drives G GPUs from this one process: each
// copies its column shard of the batch over its own PCIe link (bk_group_*).
func (krumval *KRUMValidator) initialize() {
	if bkCtx != nil {
		return
	}
	if g, err := strconv.Atoi(os.Getenv("BK_GPUS")); err == nil && g > 1 {
		var grp *C.bk_group
		if st := C.bk_group_create(&grp, C.int(g), nil, C.BK_GROUP_ALLREDUCE); st != C.BK_OK {
			outLog.Printf("bk_group_create(%d) failed (%d): %s", g, int(st),
				C.GoString(C.bk_last_error()))
			return
		}
		bkGroup, bkCtx = grp, C.bk_group_ctx(grp, 0)
		outLog.Printf("Krum engine: libbk ABI %d on %d GPUs", int(C.bk_abi_version()), g)
		return
	}
	var ctx *C.bk_ctx
	if st := C.bk_create(&ctx, 0); st != C.BK_OK {
		outLog.Printf("bk_create failed (%d): %s", int(st), C.GoString(C.bk_last_error()))
		return
	}
	bkCtx = ctx
	outLog.Printf("Krum engine: libbk ABI %d", int(C.bk_abi_version()))
}

// getTopKRUMIndex keeps the signature and the clip rule of krum.go:100-166:
// adversaryCount := int(NumAdversaries * float64(n)); the accepted indices
// index the (SourceID-sorted) UpdateList.  They come back ascending -- the
// reference returned numpy argpartition order, and its only consumer,
// checkIfAccepted, tests membership.  On any engine error every update is
// rejected (empty list), which is what a failing Python call led to.
//
// The rows go to libbk as they are (bk_multikrum_rows): a C array of the n
// row pointers, each row's backing array pinned for the call -- Go pointers
// stored in C memory, legal while pinned (runtime.Pinner, Go >= 1.21).  libbk
// packs them into its own pinned memory on host threads, each column chunk's
// H2D and Gram starting as soon as it is packed, instead of this goroutine
// copying all n rows into a pinned batch first (the old serial pack, kept
// for the multi-GPU group below).
func (krumval *KRUMValidator) getTopKRUMIndex(deltas [][]float64) []int {
	n := len(deltas)
	if n == 0 || bkCtx == nil {
		return []int{}
	}
	d := len(deltas[0])
	f := int(krumval.NumAdversaries * float64(n))
	if C.bk_check_args(C.int64_t(n), C.int64_t(d), C.int64_t(f)) != C.BK_OK {
		outLog.Printf("Krum: %s", C.GoString(C.bk_last_error()))
		return []int{}
	}
	for i := 0; i < n; i++ {
		if len(deltas[i]) != d {
			outLog.Printf("Krum: ragged update %d (%d != %d)", i, len(deltas[i]), d)
			return []int{}
		}
	}
	m := n - f
	sel := make([]C.int64_t, m)
	var mOut C.int64_t
	var st C.int
	if bkGroup != nil {
		st = groupTopKRUM(deltas, n, d, f, sel, &mOut)
	} else {
		var pinner runtime.Pinner
		defer pinner.Unpin()
		var rowsC unsafe.Pointer
		rowsC = C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(uintptr(0))))
		defer C.free(rowsC)
		ptrs := unsafe.Slice((*unsafe.Pointer)(rowsC), n)
		for i := 0; i < n; i++ {
			pinner.Pin(&deltas[i][0])
			ptrs[i] = unsafe.Pointer(&deltas[i][0])
		}
		st = C.bk_multikrum_rows(bkCtx, (*unsafe.Pointer)(rowsC), C.BK_F64, C.int64_t(n),
			C.int64_t(d), C.int64_t(f), (*C.int64_t)(unsafe.Pointer(&sel[0])), &mOut, nil, nil)
	}
	if st != C.BK_OK {
		outLog.Printf("Krum failed (%d): %s", int(st), C.GoString(C.bk_last_error()))
		return []int{}
	}
	logMargin()
	out := make([]int, int(mOut))
	for i := range out {
		out[i] = int(sel[i])
	}
	return out
}

// groupTopKRUM: BK_GPUS > 1 -- the rows packed into the C-owned pinned batch
// (serially, on this goroutine), then bk_group_multikrum, each GPU copying its
// column shard over its own PCIe link.
func groupTopKRUM(deltas [][]float64, n, d, f int, sel []C.int64_t, mOut *C.int64_t) C.int {
	need := int64(n) * int64(d) * 8
	if need > bkStageLen {
		if bkStage != nil {
			C.bk_stage_free(bkCtx, bkStage)
		}
		var p unsafe.Pointer
		if st := C.bk_stage_alloc(bkCtx, C.int64_t(need), &p); st != C.BK_OK {
			bkStage, bkStageLen = nil, 0
			return st
		}
		bkStage, bkStageLen = p, need
	}
	// pack [][]float64 rows into the pinned C buffer (row-major n x d)
	stage := unsafe.Slice((*float64)(bkStage), n*d)
	for i := 0; i < n; i++ {
		copy(stage[i*d:(i+1)*d], deltas[i])
	}
	return C.bk_group_multikrum(bkGroup, bkStage, C.BK_HOST_PINNED, C.BK_F64, C.int64_t(n),
		C.int64_t(d), C.int64_t(d), C.int64_t(f), (*C.int64_t)(unsafe.Pointer(&sel[0])), mOut,
		nil, nil)
}

// getTopKRUMIndexNoised is the same verifier call for updates that carry Delta
// and the averaged Noise vector separately (update.go:13-22; NoisedDelta =
// Delta + Noise at main.go:1524-1537): the noise is added on the GPU while the
// batch crosses PCIe (bk_multikrum_noised, SURVEY.md §8(f) row 3), so the
// verifier never builds NoisedDelta on the host.  k = 1 (Noise is already the
// mean over the noisers, main.go:1606-1653), which is bitwise Delta[i] +
// Noise[i]; updates without noise (-np=false) go with k = 0.  A batch that
// mixes the two falls back to getTopKRUMIndex over NoisedDelta.
func (krumval *KRUMValidator) getTopKRUMIndexNoised(updates []Update) []int {
	n := len(updates)
	if n == 0 || bkCtx == nil || bkGroup != nil {
		return krumval.getTopKRUMIndex(noisedDeltas(updates))
	}
	d := len(updates[0].Delta)
	k := 0
	if len(updates[0].Noise) > 0 {
		k = 1
	}
	for i := range updates {
		if len(updates[i].Delta) != d || len(updates[i].Noise) != k*d {
			return krumval.getTopKRUMIndex(noisedDeltas(updates))
		}
	}
	f := int(krumval.NumAdversaries * float64(n))
	if C.bk_check_args(C.int64_t(n), C.int64_t(d), C.int64_t(f)) != C.BK_OK {
		outLog.Printf("Krum: %s", C.GoString(C.bk_last_error()))
		return []int{}
	}
	need := int64(n) * int64(d) * 8 * int64(1+k)
	if need > bkStageLen {
		if bkStage != nil {
			C.bk_stage_free(bkCtx, bkStage)
		}
		var p unsafe.Pointer
		if C.bk_stage_alloc(bkCtx, C.int64_t(need), &p) != C.BK_OK {
			outLog.Printf("Krum: %s", C.GoString(C.bk_last_error()))
			bkStage, bkStageLen = nil, 0
			return []int{}
		}
		bkStage, bkStageLen = p, need
	}
	// pinned staging: Delta rows, then (k = 1) the Noise rows
	stage := unsafe.Slice((*float64)(bkStage), n*d*(1+k))
	for i := 0; i < n; i++ {
		copy(stage[i*d:(i+1)*d], updates[i].Delta)
		if k == 1 {
			copy(stage[(n+i)*d:(n+i+1)*d], updates[i].Noise)
		}
	}
	var noise *C.double
	if k == 1 {
		noise = (*C.double)(unsafe.Pointer(&stage[n*d]))
	}
	m := n - f
	sel := make([]C.int64_t, m)
	var mOut C.int64_t
	st := C.bk_multikrum_noised(bkCtx, (*C.double)(bkStage), C.int64_t(d), noise, C.int64_t(k),
		C.int64_t(d), C.BK_HOST_PINNED, C.int64_t(n), C.int64_t(d), C.int64_t(f),
		(*C.int64_t)(unsafe.Pointer(&sel[0])), &mOut, nil, nil, nil, 0)
	if st != C.BK_OK {
		outLog.Printf("Krum failed (%d): %s", int(st), C.GoString(C.bk_last_error()))
		return []int{}
	}
	logMargin()
	out := make([]int, int(mOut))
	for i := range out {
		out[i] = int(sel[i])
	}
	return out
}

// logMargin reports a selection the reference could legitimately make
// differently (bk_selection_margin): the boundary gap between the highest
// selected and the lowest rejected score is within the rounding bound of the
// scores, or an exact tie (k = n-f-2 = 0 makes every score 0, as on the
// localTest.sh n = 4 verifier).  Otherwise numpy's argpartition over its own
// BLAS-rounded scores (logistic_validator.py:45,59-63) provably picks the same set.
func logMargin() {
	var gap, bound C.double
	var near C.int
	if C.bk_selection_margin(bkCtx, &gap, &bound, &near) == C.BK_OK && near != 0 {
		outLog.Printf("Krum: near tie at the selection boundary (gap %g <= bound %g); "+
			"ties resolved to the lower index", float64(gap), float64(bound))
	}
}

func noisedDeltas(updates []Update) [][]float64 {
	deltas := make([][]float64, len(updates))
	for i := range updates {
		deltas[i] = updates[i].NoisedDelta
	}
	return deltas
}
