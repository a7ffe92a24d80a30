// NOT BUILT HERE: this image has no Go toolchain. This file is the reference-side binding a
// bobg/bs maintainer adds as split/gpusplit.go (package split) to drive libbsgpu through cgo;
// INTEGRATION.md §2 quotes it. It replaces hashsplit.Splitter inside split.Writer
// (split/split.go:85-90) with the GPU chunker; TreeBuilder, F and the Stores are unchanged,
// except that F hands a chunk's GPU-computed ref to stores that accept one (RefPutter) instead
// of letting st.Put hash it again. Every chunk is Put exactly once, inside F, as in
// split/split.go:71-77.

package split

/*
#cgo CFLAGS: -I${SRCDIR}/../third_party/bsgpu/include
#cgo LDFLAGS: -L${SRCDIR}/../third_party/bsgpu/lib -lbsgpu -Wl,-rpath,${SRCDIR}/../third_party/bsgpu/lib
#include <stdlib.h>
#include "bsgpu.h"
*/
import "C"

import (
	"context"
	"io"
	"math"
	"unsafe"

	"github.com/bobg/hashsplit"
	"github.com/pkg/errors"

	"github.com/bobg/bs"
)

var _ io.WriteCloser = (*GPUWriter)(nil)

// RefPutter is implemented by stores that accept a ref computed elsewhere (here: by the GPU
// chunker), in the style of bs.MultiPutter (store.go:44-47). A store that does not implement
// it gets st.Put, which computes the ref itself.
type RefPutter interface {
	PutWithRef(ctx context.Context, ref bs.Ref, b bs.Blob) (added bool, err error)
}

// bsgError maps a negative BSG_* code to a Go error; BSG_ENOTFOUND becomes bs.ErrNotFound
// (store.go:63) so callers' errors.Is checks keep working.
func bsgError(what string, rc C.int) error {
	if rc == C.BSG_ENOTFOUND {
		return bs.ErrNotFound
	}
	return errors.Errorf("%s: %s (bsgpu %d)", what, C.GoString(C.bsg_errstr(rc)), int(rc))
}

// InitGPU does libbsgpu's once-per-process start-up (device context, pooled HIP streams, copy
// engines, kernels) up front, e.g. from a server's main. Optional: the first GPUWriter pays it
// otherwise.
func InitGPU(device int) error {
	if rc := C.bsg_init(C.int(device)); rc != 0 {
		return bsgError("bsg_init", rc)
	}
	return nil
}

// GPUWriter is split.Writer (split/split.go:30-37) with the chunker and the chunk refs computed
// on an MI355X: Write / Close / Root behave as split.Writer's, and Root is bit-identical.
type GPUWriter struct {
	Ctx    context.Context
	Root   bs.Ref // populated by Close
	st     bs.Store
	rp     RefPutter // st, when it takes precomputed refs
	tb     *hashsplit.TreeBuilder
	fanout uint
	gctx   *C.bsg_ctx
	pieces []piece // stream bytes not yet emitted as chunks, oldest first
	end    uint64  // stream offset one past the last byte written
	out    []C.bsg_chunk
	// GPU refs of the chunks handed to tb.Add and not yet Put by F, keyed by the chunk's first
	// byte (chunks are disjoint, non-empty ranges of the stream, so the key is unique)
	refs map[*byte]bs.Ref
}

// piece is a run of stream bytes in a fixed Go array: appended to within its capacity only,
// never rewritten, never moved.
type piece struct {
	buf  []byte
	base uint64 // stream offset of buf[0]
}

const pieceSize = 4 << 20

// NewGPUWriter is split.NewWriter (split/split.go:44-96) on device `device`; opts are the
// reference's own Bits / MinSize / Fanout options.
func NewGPUWriter(ctx context.Context, st bs.Store, device int, opts ...Option) (*GPUWriter, error) {
	// The options are applied to a split.Writer exactly as NewWriter does, and their values
	// read back from it, so Bits / MinSize / Fanout mean what they mean there.
	ref := NewWriter(ctx, st, opts...)
	bits, minSize := ref.spl.SplitBits, ref.spl.MinSize
	p := C.bsg_params_default()
	// split.Bits / split.MinSize accept any value (split/split.go:137-152): Bits above 32 never
	// split (clamped to the C field), MinSize <= 0 is hashsplit's default (0 on the C side).
	if bits > math.MaxUint32 {
		bits = math.MaxUint32
	}
	if minSize < 0 {
		minSize = 0
	}
	if minSize > math.MaxUint32 {
		minSize = math.MaxUint32
	}
	p.split_bits, p.min_size, p.fanout = C.uint32_t(bits), C.uint32_t(minSize), C.uint32_t(ref.fanout)
	var cerr C.int
	g := C.bsg_open(C.int(device), &p, nil, &cerr)
	if g == nil {
		return nil, bsgError("bsg_open", cerr)
	}
	w := &GPUWriter{
		Ctx:    ctx,
		st:     st,
		fanout: ref.fanout,
		gctx:   g,
		out:    make([]C.bsg_chunk, 4096),
		refs:   make(map[*byte]bs.Ref),
	}
	w.rp, _ = st.(RefPutter)
	w.tb = w.newTreeBuilder()
	return w, nil
}

// newTreeBuilder is the TreeBuilder of split.NewWriter (split/split.go:51-82), except that a
// chunk whose ref the GPU computed goes to PutWithRef when the store takes refs. Either way
// every chunk is Put once, here, in the order split.Writer puts it.
func (w *GPUWriter) newTreeBuilder() *hashsplit.TreeBuilder {
	return &hashsplit.TreeBuilder{
		F: func(n *hashsplit.TreeBuilderNode) (hashsplit.Node, error) {
			var (
				offset = n.Offset()
				result = Node{
					Offset: offset,
					Size:   n.Size(),
				}
			)

			for _, child := range n.Nodes {
				childNodeWrapper := child.(*nodeWrapper)
				ref, _, err := bs.PutProto(w.Ctx, w.st, childNodeWrapper.node)
				if err != nil {
					return nil, err
				}
				result.Nodes = append(result.Nodes, &Child{Ref: ref[:], Offset: offset})
				offset += childNodeWrapper.Size()
			}

			for _, chunk := range n.Chunks {
				var (
					ref bs.Ref
					err error
				)
				gref, ok := w.refs[&chunk[0]]
				delete(w.refs, &chunk[0])
				if ok && w.rp != nil {
					ref = gref
					_, err = w.rp.PutWithRef(w.Ctx, ref, chunk) // no second hash
				} else {
					ref, _, err = w.st.Put(w.Ctx, chunk) // split/split.go:72
				}
				if err != nil {
					return nil, err
				}
				result.Leaves = append(result.Leaves, &Child{Ref: ref[:], Offset: offset})
				offset += uint64(len(chunk))
			}

			return &nodeWrapper{node: &result, ctx: w.Ctx, st: w.st}, nil
		},
	}
}

// Write implements io.Writer. bsg_write copies p into pinned staging before it returns, so no
// Go pointer is retained by C and the caller may reuse p at once.
func (w *GPUWriter) Write(p []byte) (int, error) {
	if w.tb == nil {
		return 0, errors.New("write after close")
	}
	if len(p) == 0 {
		return 0, nil
	}
	if rc := C.bsg_write(w.gctx, (*C.uint8_t)(unsafe.Pointer(&p[0])), C.size_t(len(p))); rc != 0 {
		return 0, bsgError("bsg_write", rc)
	}
	for rest := p; len(rest) > 0; {
		n := len(w.pieces)
		if n == 0 || len(w.pieces[n-1].buf) == cap(w.pieces[n-1].buf) {
			size := pieceSize
			if len(rest) > size {
				size = len(rest)
			}
			w.pieces = append(w.pieces, piece{buf: make([]byte, 0, size), base: w.end})
			n++
		}
		pc := &w.pieces[n-1]
		k := cap(pc.buf) - len(pc.buf)
		if k > len(rest) {
			k = len(rest)
		}
		pc.buf = append(pc.buf, rest[:k]...) // within capacity: the array never moves
		rest = rest[k:]
		w.end += uint64(k)
	}
	return len(p), w.drain()
}

// chunkBytes returns stream bytes [off, off+n): a full slice expression of the piece holding
// them (no copy), or, for a chunk spanning pieces, a fresh array.
func (w *GPUWriter) chunkBytes(off, n uint64) []byte {
	i := 0
	for w.pieces[i].base+uint64(len(w.pieces[i].buf)) <= off {
		i++
	}
	if lo := off - w.pieces[i].base; lo+n <= uint64(len(w.pieces[i].buf)) {
		return w.pieces[i].buf[lo : lo+n : lo+n] // cap = len: the store owns exactly these bytes
	}
	b := make([]byte, 0, n)
	for ; uint64(len(b)) < n; i++ {
		pc := w.pieces[i]
		lo := off + uint64(len(b)) - pc.base
		hi := uint64(len(pc.buf))
		if hi-lo > n-uint64(len(b)) {
			hi = lo + n - uint64(len(b))
		}
		b = append(b, pc.buf[lo:hi]...)
	}
	return b
}

// drain hands every finished chunk to the TreeBuilder in stream order, as the Splitter's
// callback does (split/split.go:85-87); F Puts it.
func (w *GPUWriter) drain() error {
	for {
		n := int(C.bsg_drain(w.gctx, &w.out[0], C.size_t(len(w.out))))
		if n == 0 {
			return nil
		}
		for _, c := range w.out[:n] {
			chunk := w.chunkBytes(uint64(c.offset), uint64(c.len))
			w.refs[&chunk[0]] = *(*bs.Ref)(unsafe.Pointer(&c.ref[0]))
			if err := w.tb.Add(chunk, uint(c.level)/w.fanout); err != nil {
				return err
			}
			// drop full pieces whose bytes are all emitted (stored chunks keep theirs alive)
			emitted := uint64(c.offset + c.len)
			for len(w.pieces) > 0 {
				pc := w.pieces[0]
				if len(pc.buf) < cap(pc.buf) || pc.base+uint64(len(pc.buf)) > emitted {
					break
				}
				w.pieces[0] = piece{}
				w.pieces = w.pieces[1:]
			}
		}
	}
}

// Close implements io.Closer: the final chunk, then the root, as split.Writer.Close does.
func (w *GPUWriter) Close() error {
	if w.tb == nil {
		return nil
	}
	if w.gctx == nil {
		return errors.New("close after a failed close")
	}
	defer func() {
		C.bsg_free(w.gctx)
		w.gctx = nil
	}()
	if rc := C.bsg_close(w.gctx); rc != 0 {
		return bsgError("bsg_close", rc)
	}
	if err := w.drain(); err != nil {
		return err
	}
	return w.closeTree()
}

// closeTree is split.Writer.Close after spl.Close (split/split.go:112-125): TreeBuilder.Root,
// then PutProto of the root node. An empty stream leaves Root at bs.Zero.
func (w *GPUWriter) closeTree() error {
	root, err := w.tb.Root()
	if err != nil {
		return err
	}
	if root != nil {
		rootNodeWrapper := root.(*nodeWrapper)
		rootRef, _, err := bs.PutProto(w.Ctx, w.st, rootNodeWrapper.node)
		if err != nil {
			return err
		}
		w.Root = rootRef
	}
	w.tb = nil
	return nil
}
