//go:build rsgpu

// Diff-checks the GPU driver against the reference CPU path (klauspost v1.12.1
// configured as in ec.go:26) on the same inputs -- the test to run on any host
// that has Go, the klauspost module and an MI355X.  (Not run in this repo's image:
// no Go toolchain.)
package ec

import (
	"bytes"
	"math/rand"
	"runtime"
	"testing"

	"github.com/klauspost/reedsolomon"

	"hybrid_distributed_store/internal/config"
)

func TestGPUMatchesReferenceCPU(t *testing.T) {
	ref, err := reedsolomon.New(config.K, config.M, reedsolomon.WithAutoGoroutines(runtime.NumCPU()))
	if err != nil {
		t.Fatal(err)
	}
	gpu := NewService()
	rng := rand.New(rand.NewSource(0x5EED0002))
	for _, n := range []int{1, 2, 3, 10, 410, 4096, 65536, 1 << 20} {
		data := make([]byte, n)
		rng.Read(data)
		want, _ := ref.Split(append([]byte(nil), data...))
		if err := ref.Encode(want); err != nil {
			t.Fatal(err)
		}
		got, err := gpu.Split(append([]byte(nil), data...))
		if err != nil {
			t.Fatal(err)
		}
		if err := gpu.Encode(got); err != nil {
			t.Fatal(err)
		}
		for i := range want {
			if !bytes.Equal(got[i], want[i]) {
				t.Fatalf("len %d shard %d differs from klauspost", n, i)
			}
		}
		for a := 0; a < 6; a++ {
			for b := a; b < 6; b++ {
				sh := make([][]byte, 6)
				copy(sh, got)
				sh[a], sh[b] = nil, nil
				if err := gpu.Reconstruct(sh); err != nil {
					t.Fatal(err)
				}
				for i := range want {
					if !bytes.Equal(sh[i], want[i]) {
						t.Fatalf("len %d erase {%d,%d}: shard %d differs", n, a, b, i)
					}
				}
			}
		}
	}
}

// The same contract on a host with no GPU: NewService must not fail and must give
// klauspost's own bytes (it IS klauspost there).  Run with HIP_VISIBLE_DEVICES=-1
// (or ROCR_VISIBLE_DEVICES=-1) to hide the GPUs.
func TestNoGPUFallsBackToKlauspost(t *testing.T) {
	if testing.Short() {
		t.Skip()
	}
	svc, ok := NewService().(*Service)
	if !ok {
		t.Fatal("NewService must return *Service")
	}
	if svc.cpu == nil {
		t.Skip("a GPU is visible; hide it to exercise the fallback")
	}
	ref, _ := reedsolomon.New(config.K, config.M)
	data := bytes.Repeat([]byte("A"), 1500*1024) // go-ycsb's hybridstore payload shape
	want, _ := ref.Split(append([]byte(nil), data...))
	_ = ref.Encode(want)
	got, err := svc.Split(append([]byte(nil), data...))
	if err != nil {
		t.Fatal(err)
	}
	if err := svc.Encode(got); err != nil {
		t.Fatal(err)
	}
	for i := range want {
		if !bytes.Equal(got[i], want[i]) {
			t.Fatalf("shard %d differs", i)
		}
	}
}
