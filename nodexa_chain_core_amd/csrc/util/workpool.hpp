// A persistent fork-join pool for the host's data-parallel loops (header batches: block proofs,
// median time past, DGW; batch packing). The previous loops spawned and joined up to 16 threads
// per call, ~10-30 us each, several times per header batch; the pool's workers stay parked on a
// condition variable between calls. One parallel_for runs at a time (others wait); a call made
// from inside a worker runs inline, so nesting cannot deadlock.
#pragma once

#include <cstddef>
#include <functional>

namespace nodexa {

// fn(lo, hi) over contiguous chunks of [0, n); at most `max_threads` participants (0 = the pool
// size: min(16, hardware threads)); ranges shorter than `min_chunk` run on the caller alone.
void parallel_for_range(size_t n, const std::function<void(size_t, size_t)>& fn, size_t min_chunk = 64,
                        size_t max_threads = 0);

template <class F>
void parallel_for_each(size_t n, F&& fn, size_t min_chunk = 64) {
    parallel_for_range(n, [&fn](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; ++i) fn(i);
    }, min_chunk);
}

size_t workpool_size();

}  // namespace nodexa
