/* Per-XCD L2 model for workgroup -> XCD orders (tools/l2_model.py).
 *
 * Each XCD is an independent set-associative LRU cache (sets x ways lines).
 * Workgroup j of the grid runs on XCD j % nxcd (round-robin dispatch, checked
 * per box by tools/xcd_map_probe.hip); an XCD keeps `slots` workgroups in
 * flight and issues one access per in-flight workgroup per step, refilling a
 * slot from its queue (grid order) when a workgroup ends.  order[j] is the
 * block workgroup j runs; block b's accesses are lines[off[b] .. off[b+1])
 * with a class id each.  Out: hits[c], misses[c] summed over XCDs.
 * CPU-only model; build: gcc -O2 -shared -fPIC l2sim.c -o l2sim.so */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

int l2sim(int64_t n_blocks, const int32_t *order, int nxcd, int slots, const int64_t *off,
          const uint64_t *lines, const uint8_t *cls, int sets, int ways, int ncls, int64_t *hits,
          int64_t *misses) {
  uint64_t *tag = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)sets * ways);
  uint64_t *age = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)sets * ways);
  int64_t *cur = (int64_t *)malloc(sizeof(int64_t) * slots);
  int64_t *end = (int64_t *)malloc(sizeof(int64_t) * slots);
  if (!tag || !age || !cur || !end) return -1;
  memset(hits, 0, sizeof(int64_t) * ncls);
  memset(misses, 0, sizeof(int64_t) * ncls);
  for (int xcd = 0; xcd < nxcd; ++xcd) {
    for (int64_t i = 0; i < (int64_t)sets * ways; ++i) {
      tag[i] = ~0ull;
      age[i] = 0;
    }
    uint64_t clock = 1;
    int64_t next = xcd;  // next grid index of this XCD
    int live = 0;
    for (int s = 0; s < slots; ++s) {
      cur[s] = end[s] = 0;
      if (next < n_blocks) {
        const int32_t b = order[next];
        cur[s] = off[b];
        end[s] = off[b + 1];
        next += nxcd;
        ++live;
      }
    }
    while (live > 0) {
      for (int s = 0; s < slots; ++s) {
        if (cur[s] >= end[s]) continue;
        const uint64_t ln = lines[cur[s]];
        const int c = cls[cur[s]];
        ++cur[s];
        const uint64_t h = ln ^ (ln >> 11) ^ (ln >> 22);
        const int64_t set = (int64_t)(h % (uint64_t)sets);
        uint64_t *t = tag + set * ways, *a = age + set * ways;
        int w = 0, hit = 0;
        for (int k = 0; k < ways; ++k)
          if (t[k] == ln) {
            w = k;
            hit = 1;
            break;
          }
        if (!hit) {
          uint64_t oldest = ~0ull;
          for (int k = 0; k < ways; ++k)
            if (a[k] < oldest) {
              oldest = a[k];
              w = k;
            }
          t[w] = ln;
        }
        a[w] = clock++;
        if (hit)
          ++hits[c];
        else
          ++misses[c];
        if (cur[s] >= end[s]) {
          if (next < n_blocks) {
            const int32_t b = order[next];
            cur[s] = off[b];
            end[s] = off[b + 1];
            next += nxcd;
          } else {
            --live;
          }
        }
      }
    }
  }
  free(tag);
  free(age);
  free(cur);
  free(end);
  return 0;
}
