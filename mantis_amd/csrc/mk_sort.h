// getBestNHypotheses (include/mantis3/HypothesisEvaluation.h:484-518) sorts
// hypotheses with std::sort(wayToSort), an unstable sort, and keeps the tail:
// which of several equal-error hypotheses survives depends on libstdc++'s
// introsort. This is that algorithm (GCC 5-13 bits/stl_algo.h + stl_heap.h:
// median-of-three pivot, unguarded partition, depth limit 2*floor(log2 n),
// heapsort fallback, threshold-16 final insertion sort), restated for one
// work-item over an array of {error, index} records, so the device keeps the
// same survivor the reference would.
#pragma once
#include "mk_math.h"

namespace mk {

struct ErrIdx {
  double e;
  int i;
};

// wayToSort(i, j) = j.error < i.error (descending)
MK_HD bool way_to_sort(const ErrIdx& a, const ErrIdx& b) { return b.e < a.e; }

MK_HD void ei_swap(ErrIdx* a, ErrIdx* b) { ErrIdx t = *a; *a = *b; *b = t; }

MK_HD void heap_push(ErrIdx* first, long hole, long top, ErrIdx value) {
  long parent = (hole - 1) / 2;
  while (hole > top && way_to_sort(first[parent], value)) {
    first[hole] = first[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  first[hole] = value;
}
MK_HD void heap_adjust(ErrIdx* first, long hole, long len, ErrIdx value) {
  const long top = hole;
  long second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (way_to_sort(first[second], first[second - 1])) second--;
    first[hole] = first[second];
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    first[hole] = first[second - 1];
    hole = second - 1;
  }
  heap_push(first, hole, top, value);
}
MK_HD void heap_make(ErrIdx* first, ErrIdx* last) {
  long len = last - first;
  if (len < 2) return;
  long parent = (len - 2) / 2;
  while (true) {
    ErrIdx v = first[parent];
    heap_adjust(first, parent, len, v);
    if (parent == 0) return;
    parent--;
  }
}
MK_HD void heap_pop(ErrIdx* first, ErrIdx* last, ErrIdx* result) {
  ErrIdx v = *result;
  *result = *first;
  heap_adjust(first, 0, last - first, v);
}
MK_HD void partial_sort_all(ErrIdx* first, ErrIdx* last) {
  heap_make(first, last);  // __heap_select(first, last, last)
  while (last - first > 1) {
    --last;
    heap_pop(first, last, last);
  }
}
MK_HD void move_median_to_first(ErrIdx* result, ErrIdx* a, ErrIdx* b, ErrIdx* c) {
  if (way_to_sort(*a, *b)) {
    if (way_to_sort(*b, *c)) ei_swap(result, b);
    else if (way_to_sort(*a, *c)) ei_swap(result, c);
    else ei_swap(result, a);
  } else if (way_to_sort(*a, *c)) {
    ei_swap(result, a);
  } else if (way_to_sort(*b, *c)) {
    ei_swap(result, c);
  } else {
    ei_swap(result, b);
  }
}
MK_HD ErrIdx* unguarded_partition(ErrIdx* first, ErrIdx* last, ErrIdx* pivot) {
  while (true) {
    while (way_to_sort(*first, *pivot)) ++first;
    --last;
    while (way_to_sort(*pivot, *last)) --last;
    if (!(first < last)) return first;
    ei_swap(first, last);
    ++first;
  }
}
MK_HD void introsort_loop(ErrIdx* first, ErrIdx* last, int depth_limit) {
  // iterative form of the reference recursion: recurse on the right part,
  // loop on the left part (same visiting order, explicit stack)
#if MK_DM_DEVICE
  // one thread per block sorts (k_score_init / k_score_final, tid 0): the
  // explicit stack lives in LDS instead of 1.3 KB of per-lane scratch that
  // every lane of those kernels would otherwise be allocated
  __shared__ ErrIdx* st_first[64];
  __shared__ ErrIdx* st_last[64];
  __shared__ int st_depth[64];
#else
  ErrIdx* st_first[64];
  ErrIdx* st_last[64];
  int st_depth[64];
#endif
  int sp = 0;
  st_first[sp] = first; st_last[sp] = last; st_depth[sp] = depth_limit; sp++;
  while (sp > 0) {
    sp--;
    first = st_first[sp]; last = st_last[sp]; depth_limit = st_depth[sp];
    while (last - first > 16) {
      if (depth_limit == 0) {
        partial_sort_all(first, last);
        break;
      }
      --depth_limit;
      ErrIdx* mid = first + (last - first) / 2;
      move_median_to_first(first, first + 1, mid, last - 1);
      ErrIdx* cut = unguarded_partition(first + 1, last, first);
      // std::__introsort_loop(cut, last, depth) runs to completion before the
      // loop continues on [first, cut): push the left part, process the right now.
      st_first[sp] = first; st_last[sp] = cut; st_depth[sp] = depth_limit; sp++;
      first = cut;
    }
  }
}
MK_HD void unguarded_linear_insert(ErrIdx* last) {
  ErrIdx val = *last;
  ErrIdx* next = last - 1;
  while (way_to_sort(val, *next)) {
    *last = *next;
    last = next;
    --next;
  }
  *last = val;
}
MK_HD void insertion_sort(ErrIdx* first, ErrIdx* last) {
  if (first == last) return;
  for (ErrIdx* i = first + 1; i != last; ++i) {
    if (way_to_sort(*i, *first)) {
      ErrIdx val = *i;
      for (ErrIdx* k = i; k != first; --k) *k = *(k - 1);
      *first = val;
    } else {
      unguarded_linear_insert(i);
    }
  }
}
MK_HD int lg2(long n) {
  int r = 0;
  while (n > 1) { n >>= 1; r++; }
  return r;
}
MK_HD void std_sort_desc(ErrIdx* first, ErrIdx* last) {
  if (first == last) return;
  introsort_loop(first, last, lg2(last - first) * 2);
  if (last - first > 16) {
    insertion_sort(first, first + 16);
    for (ErrIdx* i = first + 16; i != last; ++i) unguarded_linear_insert(i);
  } else {
    insertion_sort(first, last);
  }
}

}  // namespace mk
