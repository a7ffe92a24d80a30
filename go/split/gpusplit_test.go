// NOT BUILT HERE: this image has no Go toolchain. Tests for go/split/gpusplit.go, to sit
// beside the reference's split/split_test.go: its two tests (split_test.go:15-108) run on the
// GPUWriter, and the GPUWriter's Root and stored blobs are compared with split.Writer's on the
// same bytes — the Go-pinned parity check this repository's oracle cannot run without Go
// (DESIGN.md §2; tests/golden/tree_root_variants.json holds streams where a recalled tree
// detail would show).

package split

import (
	"bytes"
	"context"
	"io"
	"math/rand"
	"os"
	"testing"
	"testing/quick"

	"github.com/bobg/bs"
	"github.com/bobg/bs/store/mem"
)

func TestGPUSplitEmpty(t *testing.T) { // split_test.go:15-25
	m := mem.New()
	w, err := NewGPUWriter(context.Background(), m, 0)
	if err != nil {
		t.Fatal(err)
	}
	if err = w.Close(); err != nil {
		t.Fatal(err)
	}
	if w.Root != bs.Zero {
		t.Errorf("got Root of %s, want %s", w.Root, bs.Zero)
	}
}

func TestGPUSplit(t *testing.T) { // split_test.go:27-108
	var (
		ctx = context.Background()
		s   = mem.New()
	)
	w, err := NewGPUWriter(ctx, s, 0, Bits(4), Fanout(2))
	if err != nil {
		t.Fatal(err)
	}
	f, err := os.Open("../testdata/yubnub.opus")
	if err != nil {
		t.Fatal(err)
	}
	defer f.Close()
	if _, err = io.Copy(w, f); err != nil {
		t.Fatal(err)
	}
	if err = w.Close(); err != nil {
		t.Fatal(err)
	}
	max, err := f.Seek(0, io.SeekEnd)
	if err != nil {
		t.Fatal(err)
	}
	r, err := NewReader(ctx, s, w.Root)
	if err != nil {
		t.Fatal(err)
	}
	err = quick.Check(func(offset int64, nbytes int) bool {
		offset %= max
		if offset < 0 {
			offset = -offset
		}
		if nbytes < 0 {
			nbytes = 1
		}
		if offset+int64(nbytes) > max {
			nbytes = int(max - offset)
		}
		want, got := make([]byte, nbytes), make([]byte, nbytes)
		if _, err := f.Seek(offset, io.SeekStart); err != nil {
			return false
		}
		if _, err := f.Read(want); err != nil {
			return false
		}
		if _, err := r.Seek(offset, io.SeekStart); err != nil {
			return false
		}
		if _, err := r.Read(got); err != nil {
			return false
		}
		return bytes.Equal(got, want)
	}, nil)
	if err != nil {
		t.Error(err)
	}
}

// refs lists a store's refs in order.
func refs(t *testing.T, s bs.Getter) []bs.Ref {
	var out []bs.Ref
	if err := s.ListRefs(context.Background(), bs.Zero, func(r bs.Ref) error {
		out = append(out, r)
		return nil
	}); err != nil {
		t.Fatal(err)
	}
	return out
}

// putCounter is a store/mem that takes precomputed refs and counts every Put.
type putCounter struct {
	*mem.Store
	puts, withRef int
}

func (p *putCounter) Put(ctx context.Context, b bs.Blob) (bs.Ref, bool, error) {
	p.puts++
	return p.Store.Put(ctx, b)
}

func (p *putCounter) PutWithRef(ctx context.Context, ref bs.Ref, b bs.Blob) (bool, error) {
	p.withRef++
	if b.Ref() != ref {
		return false, bs.ErrNotFound // a wrong GPU ref fails the test below
	}
	_, added, err := p.Store.Put(ctx, b)
	return added, err
}

// TestGPUWriterMatchesWriter: the same bytes through split.Writer and GPUWriter give the same
// Root and the same stored blobs, for the reference's testdata and random streams, under
// default and edge options; with a RefPutter store every chunk is Put once, with its GPU ref.
func TestGPUWriterMatchesWriter(t *testing.T) {
	ctx := context.Background()
	var inputs [][]byte
	for _, name := range []string{"../testdata/yubnub.opus", "../testdata/commonsense.txt"} {
		b, err := os.ReadFile(name)
		if err != nil {
			t.Fatal(err)
		}
		inputs = append(inputs, b)
	}
	rng := rand.New(rand.NewSource(1))
	for _, n := range []int{0, 1, 1023, 1024, 1025, 65536, 3 << 20, 40 << 20} {
		b := make([]byte, n)
		rng.Read(b)
		inputs = append(inputs, b)
	}
	optsets := [][]Option{
		nil,
		{Bits(4), Fanout(2)},
		{Bits(10), MinSize(64), Fanout(3)},
		{Bits(20), MinSize(4096)},
	}
	for i, in := range inputs {
		for j, opts := range optsets {
			ms := mem.New()
			w := NewWriter(ctx, ms, opts...)
			if _, err := w.Write(in); err != nil {
				t.Fatal(err)
			}
			if err := w.Close(); err != nil {
				t.Fatal(err)
			}

			gs := &putCounter{Store: mem.New()}
			g, err := NewGPUWriter(ctx, gs, 0, opts...)
			if err != nil {
				t.Fatal(err)
			}
			for off := 0; off < len(in); off += 1 << 20 { // several Writes
				end := off + 1<<20
				if end > len(in) {
					end = len(in)
				}
				if _, err := g.Write(in[off:end]); err != nil {
					t.Fatal(err)
				}
			}
			if err := g.Close(); err != nil {
				t.Fatal(err)
			}
			if g.Root != w.Root {
				t.Errorf("input %d, options %d: GPU Root %s, split.Writer Root %s", i, j, g.Root, w.Root)
			}
			want, got := refs(t, ms), refs(t, gs)
			if len(want) != len(got) {
				t.Fatalf("input %d, options %d: %d blobs, want %d", i, j, len(got), len(want))
			}
			for k := range want {
				if want[k] != got[k] {
					t.Fatalf("input %d, options %d: blob %d is %s, want %s", i, j, k, got[k], want[k])
				}
			}
			if len(g.refs) != 0 {
				t.Errorf("input %d, options %d: %d GPU refs never Put", i, j, len(g.refs))
			}
			// chunks arrive with their ref (PutWithRef); only tree nodes go through Put
			if gs.withRef == 0 && len(in) > 0 {
				t.Errorf("input %d, options %d: no chunk took the PutWithRef path", i, j)
			}
		}
	}
}
