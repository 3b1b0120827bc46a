// TEST INFRASTRUCTURE ONLY (tests/ load it through oracle.py; the product path never does).
//
// The reference orders its candidates with an unstable std::sort (feature_point_detector.cpp:58-60,
// comparator: response greater). Its permutation of equal responses is libstdc++'s introsort run on the
// pushed sequence, including the heapsort fallback (std::__partial_sort) of a range that reaches the
// depth limit 2 * floor(log2 n). The GPU emulates that order (fd_select_ref.hip). This file
//   * restates libstdc++ 11's std::sort (bits/stl_algo.h __introsort_loop, __unguarded_partition_pivot,
//     __final_insertion_sort; bits/stl_heap.h __make_heap, __adjust_heap, __push_heap, __pop_heap,
//     __sort_heap) with a trace of the ranges that take the heapsort path, so the tests can check the
//     restatement against std::sort itself and know that an input reaches the fallback;
//   * builds such inputs with McIlroy's adversary ("A Killer Adversary for Quicksort", Software--Practice
//     and Experience 29(4), 1999) run against std::sort with the reference comparator: values are fixed
//     lazily as the sort compares them, so that every pivot is an extreme of the undecided ("gas")
//     elements; the gas left at the end shares one value (a run of ties).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

struct Elem {
    float resp;
    uint32_t idx;
};
// the reference comparator: a is visited before b (feature_point_detector.cpp:58-60)
struct RespGreater {
    bool operator()(const Elem &a, const Elem &b) const { return a.resp > b.resp; }
};

struct Trace {
    int64_t heap_ranges = 0;
    int64_t first_lo = -1, first_hi = -1;  // the heapsorted range nearest the front
    int64_t min_depth_left = 1 << 30;
    bool heap_seen = false;  // set once a range is heapsorted (the adversary stops fixing values then)
};

// bits/stl_heap.h
template <class T, class C>
void push_heap(T *f, int64_t hole, int64_t top, T v, C &comp) {
    int64_t parent = (hole - 1) / 2;
    while (hole > top && comp(f[parent], v)) {
        f[hole] = f[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    f[hole] = v;
}

template <class T, class C>
void adjust_heap(T *f, int64_t hole, int64_t len, T v, C &comp) {
    const int64_t top = hole;
    int64_t second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (comp(f[second], f[second - 1])) --second;
        f[hole] = f[second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        f[hole] = f[second - 1];
        hole = second - 1;
    }
    push_heap(f, hole, top, v, comp);
}

template <class T, class C>
void make_heap(T *f, int64_t len, C &comp) {
    if (len < 2) return;
    for (int64_t parent = (len - 2) / 2;; --parent) {
        adjust_heap(f, parent, len, f[parent], comp);
        if (parent == 0) return;
    }
}

template <class T, class C>
void sort_heap(T *f, int64_t len, C &comp) {
    while (len > 1) {
        --len;
        const T v = f[len];
        f[len] = f[0];
        adjust_heap(f, 0, len, v, comp);
    }
}

// bits/stl_algo.h
template <class T, class C>
void move_median_to_first(T *result, T *a, T *b, T *c, C &comp) {
    if (comp(*a, *b)) {
        if (comp(*b, *c)) std::swap(*result, *b);
        else if (comp(*a, *c)) std::swap(*result, *c);
        else std::swap(*result, *a);
    } else if (comp(*a, *c)) {
        std::swap(*result, *a);
    } else if (comp(*b, *c)) {
        std::swap(*result, *c);
    } else {
        std::swap(*result, *b);
    }
}

template <class T, class C>
T *unguarded_partition(T *first, T *last, T *pivot, C &comp) {
    while (true) {
        while (comp(*first, *pivot)) ++first;
        --last;
        while (comp(*pivot, *last)) --last;
        if (!(first < last)) return first;
        std::swap(*first, *last);
        ++first;
    }
}

template <class T, class C>
void introsort_loop(T *base, T *first, T *last, int64_t depth, C &comp, Trace &t) {
    while (last - first > 16) {
        if (depth == 0) {  // std::__partial_sort(first, last, last): __heap_select (= make_heap) + __sort_heap
            t.heap_seen = true;
            make_heap(first, last - first, comp);
            sort_heap(first, last - first, comp);
            ++t.heap_ranges;
            if (t.first_lo < 0 || first - base < t.first_lo) {
                t.first_lo = first - base;
                t.first_hi = last - base;
            }
            return;
        }
        --depth;
        t.min_depth_left = std::min(t.min_depth_left, depth);
        T *mid = first + (last - first) / 2;
        move_median_to_first(first, first + 1, mid, last - 1, comp);
        T *cut = unguarded_partition(first + 1, last, first, comp);
        introsort_loop(base, cut, last, depth, comp, t);
        last = cut;
    }
}

template <class T, class C>
void unguarded_linear_insert(T *last, C &comp) {
    const T v = *last;
    T *next = last - 1;
    while (comp(v, *next)) {
        *last = *next;
        last = next;
        --next;
    }
    *last = v;
}

template <class T, class C>
void insertion_sort(T *first, T *last, C &comp) {
    if (first == last) return;
    for (T *i = first + 1; i != last; ++i) {
        if (comp(*i, *first)) {
            const T v = *i;
            std::move_backward(first, i, i + 1);
            *first = v;
        } else {
            unguarded_linear_insert(i, comp);
        }
    }
}

template <class T, class C>
void std_sort_restated(T *first, T *last, C &comp, Trace &t) {
    if (first == last) return;
    const int64_t n = last - first;
    const int64_t lg = 63 - __builtin_clzll(static_cast<unsigned long long>(n));
    introsort_loop(first, first, last, 2 * lg, comp, t);
    if (n > 16) {
        insertion_sort(first, first + 16, comp);
        for (T *i = first + 16; i != last; ++i) unguarded_linear_insert(i, comp);
    } else {
        insertion_sort(first, last, comp);
    }
}

}  // namespace

extern "C" {

// std::sort itself on (resp[i], i): perm[k] = the index visited k-th.
void orc_std_sort_perm(const float *resp, int64_t n, uint32_t *perm) {
    std::vector<Elem> v(static_cast<size_t>(n));
    for (int64_t i = 0; i < n; ++i) v[static_cast<size_t>(i)] = {resp[i], static_cast<uint32_t>(i)};
    std::sort(v.begin(), v.end(), RespGreater());
    for (int64_t i = 0; i < n; ++i) perm[i] = v[static_cast<size_t>(i)].idx;
}

// The restatement: perm as orc_std_sort_perm; stats[0] heapsorted ranges, stats[1..2] the frontmost one
// [lo, hi) (-1 if none), stats[3] the smallest depth left after a partition.
void orc_std_sort_restated(const float *resp, int64_t n, uint32_t *perm, int64_t *stats) {
    std::vector<Elem> v(static_cast<size_t>(n));
    for (int64_t i = 0; i < n; ++i) v[static_cast<size_t>(i)] = {resp[i], static_cast<uint32_t>(i)};
    Trace t;
    RespGreater comp;
    std_sort_restated(v.data(), v.data() + n, comp, t);
    for (int64_t i = 0; i < n; ++i) perm[i] = v[static_cast<size_t>(i)].idx;
    stats[0] = t.heap_ranges;
    stats[1] = t.first_lo;
    stats[2] = t.first_hi;
    stats[3] = t.min_depth_left;
}

// McIlroy's adversary against the restated std::sort (equal to std::sort, tests/test_oracle_select.py)
// with the reference comparator. front = 1: the undecided ("gas") elements are visited first (the
// largest response) and each frozen pivot candidate takes the next value from the far end, so the
// partitions peel the back and the long range stays at the front -- the range the greedy visits first;
// front = 0: the mirror image. Values are fixed only until the heapsort fallback starts: the gas still
// undecided then keeps one value (a run of equal responses inside the heapsorted range). resp[i] = the value of element i in push order (small integers as floats, exact).
void orc_introsort_killer(int64_t n, int front, float *resp) {
    std::vector<int64_t> val(static_cast<size_t>(n));
    const int64_t gas = front ? -1 : n;  // visited first (front) / last
    for (auto &x : val) x = gas;
    int64_t nsolid = front ? n - 1 : 0;  // frozen values: from the far end towards the gas
    int64_t candidate = -1;
    Trace t;
    auto freeze = [&](int64_t x) { val[static_cast<size_t>(x)] = front ? nsolid-- : nsolid++; };
    // "a before b" = a.resp > b.resp with resp = -val
    auto before = [&](uint32_t x, uint32_t y) {
        if (!t.heap_seen) {
            if (val[x] == gas && val[y] == gas) {
                if (static_cast<int64_t>(x) == candidate) freeze(x);
                else freeze(y);
            }
            if (val[x] == gas) candidate = x;
            else if (val[y] == gas) candidate = y;
        }
        return val[x] < val[y];
    };
    std::vector<uint32_t> ix(static_cast<size_t>(n));
    for (int64_t i = 0; i < n; ++i) ix[static_cast<size_t>(i)] = static_cast<uint32_t>(i);
    std_sort_restated(ix.data(), ix.data() + n, before, t);
    for (int64_t i = 0; i < n; ++i) resp[i] = static_cast<float>(-val[static_cast<size_t>(i)]);
}

}  // extern "C"
