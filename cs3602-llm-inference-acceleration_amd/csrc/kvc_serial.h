// kvc_serial.h -- the serial pieces of libstdc++'s std::sort / std::nth_element /
// std::partial_sort, restated on a (key[], idx[]) pair of arrays (LDS in the select kernel).
//
// The selection kernel reproduces which elements libstdc++ leaves in the first k positions.
// Its block-parallel part computes Hoare partitions; the serial steps that remain -- the
// median-of-three pivot move, the final insertion sort of a <=16 (<=3) element segment, and the
// rare heap fallbacks (introsort depth limit, std::partial_sort's heap select) -- run on one
// lane and must follow the libstdc++ code exactly (bits/stl_algo.h, bits/stl_heap.h):
//   std::__move_median_to_first, std::__insertion_sort / __unguarded_linear_insert,
//   std::__adjust_heap, std::__push_heap, std::__make_heap, std::__pop_heap,
//   std::__sort_heap, std::__heap_select.
// tests/native/select_model.cpp (run by tests/test_select_model.py) checks these, with the
// kernel's own key mapping, against the real libstdc++ algorithms.
#pragma once

#include "kvc_common.h"

namespace kvc {

template <typename K, typename I>
KVC_HD void kv_swap(K* key, I* idx, int a, int b) {
  const K tk = key[a];
  key[a] = key[b];
  key[b] = tk;
  const I ti = idx[a];
  idx[a] = idx[b];
  idx[b] = ti;
}

// std::__move_median_to_first(result, a, b, c, comp) with comp = key '<'.
template <typename K, typename I>
KVC_HD void move_median_to_first(K* key, I* idx, int result, int a, int b, int c) {
  if (key[a] < key[b]) {
    if (key[b] < key[c])
      kv_swap(key, idx, result, b);
    else if (key[a] < key[c])
      kv_swap(key, idx, result, c);
    else
      kv_swap(key, idx, result, a);
  } else if (key[a] < key[c]) {
    kv_swap(key, idx, result, a);
  } else if (key[b] < key[c]) {
    kv_swap(key, idx, result, c);
  } else {
    kv_swap(key, idx, result, b);
  }
}

// Stable insertion sort of [lo, hi): the arrangement std::__insertion_sort and
// std::__unguarded_linear_insert produce (an element moves left only past strictly greater ones).
template <typename K, typename I>
KVC_HD void insertion_sort(K* key, I* idx, int lo, int hi) {
  for (int i = lo + 1; i < hi; ++i) {
    const K vk = key[i];
    const I vi = idx[i];
    int j = i;
    while (j > lo && vk < key[j - 1]) {
      key[j] = key[j - 1];
      idx[j] = idx[j - 1];
      --j;
    }
    key[j] = vk;
    idx[j] = vi;
  }
}

// std::__adjust_heap(first, hole, len, value) followed by std::__push_heap.
template <typename K, typename I>
KVC_HD void adjust_heap(K* key, I* idx, int hole, int len, K vk, I vi) {
  const int top = hole;
  int second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (key[second] < key[second - 1]) --second;
    key[hole] = key[second];
    idx[hole] = idx[second];
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    key[hole] = key[second - 1];
    idx[hole] = idx[second - 1];
    hole = second - 1;
  }
  int parent = (hole - 1) / 2;
  while (hole > top && key[parent] < vk) {
    key[hole] = key[parent];
    idx[hole] = idx[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  key[hole] = vk;
  idx[hole] = vi;
}

// std::__make_heap(first, first + len)
template <typename K, typename I>
KVC_HD void make_heap(K* key, I* idx, int len) {
  if (len < 2) return;
  int parent = (len - 2) / 2;
  while (true) {
    const K vk = key[parent];
    const I vi = idx[parent];
    adjust_heap(key, idx, parent, len, vk, vi);
    if (parent == 0) return;
    --parent;
  }
}

// std::__pop_heap(first, first + len, first + result)
template <typename K, typename I>
KVC_HD void pop_heap(K* key, I* idx, int len, int result) {
  const K vk = key[result];
  const I vi = idx[result];
  key[result] = key[0];
  idx[result] = idx[0];
  adjust_heap(key, idx, 0, len, vk, vi);
}

// std::__sort_heap(first, first + len)
template <typename K, typename I>
KVC_HD void sort_heap(K* key, I* idx, int len) {
  while (len > 1) {
    --len;
    pop_heap(key, idx, len, len);
  }
}

// std::__heap_select(first, first + middle, first + len)
template <typename K, typename I>
KVC_HD void heap_select(K* key, I* idx, int middle, int len) {
  make_heap(key, idx, middle);
  for (int i = middle; i < len; ++i)
    if (key[i] < key[0]) pop_heap(key, idx, middle, i);
}

KVC_HD int floor_log2(int n) {
  int r = 0;
  while (n > 1) {
    n >>= 1;
    ++r;
  }
  return r;
}

}  // namespace kvc
