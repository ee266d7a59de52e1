// slo_introsort.h — libstdc++ (GCC 11) std::sort, restated for one GPU lane.
//
// extractFeatures (featureAssociation.cpp:699) sorts each sector of the
// persistent cloudSmoothness array with std::sort, which is unstable: the
// order of equal curvatures — and the content left at each position, which
// persists into the next scan — is whatever
// libstdc++'s introsort produces.  This is that algorithm, step for step
// (median-of-three pivot into *first, unguarded Hoare partition, depth limit
// 2*floor(log2 n) with heapsort fallback, threshold 16, final guarded +
// unguarded insertion sort).  Disjoint sub-ranges are independent, so the
// recursion on the right part becomes an explicit stack without changing the
// result.  tests/test_introsort.py checks it against std::sort on arrays full
// of ties.
#pragma once

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define SLO_SORT_HD __host__ __device__ inline
#else
#define SLO_SORT_HD inline
#endif

namespace slo_sort {

template <class T>
SLO_SORT_HD void swap_(T& a, T& b) { T t = a; a = b; b = t; }

template <class T, class Less>
SLO_SORT_HD void push_heap_(T* first, int hole, int top, T value, Less less) {
    int parent = (hole - 1) / 2;
    while (hole > top && less(first[parent], value)) {
        first[hole] = first[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    first[hole] = value;
}

template <class T, class Less>
SLO_SORT_HD void adjust_heap_(T* first, int hole, int len, T value, Less less) {
    const int top = hole;
    int second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (less(first[second], first[second - 1])) second--;
        first[hole] = first[second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        first[hole] = first[second - 1];
        hole = second - 1;
    }
    push_heap_(first, hole, top, value, less);
}

template <class T, class Less>
SLO_SORT_HD void heap_sort_(T* first, int len, Less less) {
    if (len >= 2) {  // make_heap
        int parent = (len - 2) / 2;
        while (true) {
            T v = first[parent];
            adjust_heap_(first, parent, len, v, less);
            if (parent == 0) break;
            parent--;
        }
    }
    while (len > 1) {  // sort_heap
        --len;
        T v = first[len];
        first[len] = first[0];
        adjust_heap_(first, 0, len, v, less);
    }
}

template <class T, class Less>
SLO_SORT_HD void move_median_to_first_(T* result, T* a, T* b, T* c, Less less) {
    if (less(*a, *b)) {
        if (less(*b, *c)) swap_(*result, *b);
        else if (less(*a, *c)) swap_(*result, *c);
        else swap_(*result, *a);
    } else if (less(*a, *c)) swap_(*result, *a);
    else if (less(*b, *c)) swap_(*result, *c);
    else swap_(*result, *b);
}

template <class T, class Less>
SLO_SORT_HD T* unguarded_partition_(T* first, T* last, T* pivot, Less less) {
    while (true) {
        while (less(*first, *pivot)) ++first;
        --last;
        while (less(*pivot, *last)) --last;
        if (!(first < last)) return first;
        swap_(*first, *last);
        ++first;
    }
}

template <class T, class Less>
SLO_SORT_HD void unguarded_linear_insert_(T* last, Less less) {
    T val = *last;
    T* next = last - 1;
    while (less(val, *next)) {
        *last = *next;
        last = next;
        --next;
    }
    *last = val;
}

template <class T, class Less>
SLO_SORT_HD void insertion_sort_(T* first, T* last, Less less) {
    if (first == last) return;
    for (T* i = first + 1; i != last; ++i) {
        if (less(*i, *first)) {
            T val = *i;
            for (T* p = i; p != first; --p) *p = *(p - 1);
            *first = val;
        } else {
            unguarded_linear_insert_(i, less);
        }
    }
}

SLO_SORT_HD int lg_(int n) {
    int r = 0;
    while (n > 1) { n >>= 1; ++r; }
    return r;
}

// Sorts [first, first+n) exactly as libstdc++'s std::sort(first, first+n, less).
template <class T, class Less>
SLO_SORT_HD void std_sort(T* first, int n, Less less) {
    if (n <= 1) return;
    const int threshold = 16;
    // explicit stack of (lo, hi, depth) for the right-hand recursion
    int st_lo[64], st_hi[64], st_d[64];
    int sp = 0;
    st_lo[sp] = 0; st_hi[sp] = n; st_d[sp] = 2 * lg_(n); sp++;
    while (sp > 0) {
        sp--;
        int lo = st_lo[sp], hi = st_hi[sp], depth = st_d[sp];
        while (hi - lo > threshold) {
            if (depth == 0) {
                heap_sort_(first + lo, hi - lo, less);
                break;
            }
            --depth;
            T* f = first + lo;
            T* l = first + hi;
            T* mid = f + (hi - lo) / 2;
            move_median_to_first_(f, f + 1, mid, l - 1, less);
            T* cut = unguarded_partition_(f + 1, l, f, less);
            int c = (int)(cut - first);
            st_lo[sp] = c; st_hi[sp] = hi; st_d[sp] = depth; sp++;
            hi = c;
        }
    }
    if (n > threshold) {
        insertion_sort_(first, first + threshold, less);
        for (T* i = first + threshold; i != first + n; ++i) unguarded_linear_insert_(i, less);
    } else {
        insertion_sort_(first, first + n, less);
    }
}

// What std::sort still does to one sub-range [first, first+n) that its
// introsort loop reaches with `depth` levels of budget left: the rest of the
// loop on it, then the final insertion sort restricted to it.  The global
// final insertion sort never moves an element across a partition boundary
// (everything left of a cut is <= everything right of it, and an element
// only passes strictly greater ones), so restricting it to the sub-range —
// and making it guarded — changes nothing.  Used by the PCL-order VoxelGrid
// (slo_pclsort.h) for the sub-ranges one lane finishes.
// (st_lo / st_hi / st_d: the caller's stack of 64 entries each, e.g. LDS on
// the GPU, where a private one is 768 B of scratch memory per lane)
template <class T, class Less>
SLO_SORT_HD void introsort_range_ws(T* first, int n, int depth, Less less, int* st_lo, int* st_hi, int* st_d) {
    if (n <= 1) return;
    const int threshold = 16;
    int sp = 0;
    st_lo[sp] = 0; st_hi[sp] = n; st_d[sp] = depth; sp++;
    while (sp > 0) {
        sp--;
        int lo = st_lo[sp], hi = st_hi[sp], dep = st_d[sp];
        while (hi - lo > threshold) {
            if (dep == 0) {
                heap_sort_(first + lo, hi - lo, less);
                break;
            }
            --dep;
            T* f = first + lo;
            T* l = first + hi;
            T* mid = f + (hi - lo) / 2;
            move_median_to_first_(f, f + 1, mid, l - 1, less);
            T* cut = unguarded_partition_(f + 1, l, f, less);
            int c = (int)(cut - first);
            st_lo[sp] = c; st_hi[sp] = hi; st_d[sp] = dep; sp++;
            hi = c;
        }
    }
    insertion_sort_(first, first + n, less);
}
template <class T, class Less>
SLO_SORT_HD void introsort_range(T* first, int n, int depth, Less less) {
    int st_lo[64], st_hi[64], st_d[64];
    introsort_range_ws(first, n, depth, less, st_lo, st_hi, st_d);
}

// The two loops above for n <= 8191 (the GPU's lane tasks: PCL-sort ranges
// of an LDS finish entry, featureAssociation's sector sorts), with the stack
// packed one entry per 32-bit word (lo 13 | hi 13 | depth 6 bits): 256 B of
// private memory per lane instead of 768.  The depths on the stack strictly
// decrease from bottom to top (a push stores the decremented depth of the
// range in hand, and a popped range's pushes store less again), so it holds
// at most depth + 1 <= 64 entries.  The same steps in the same order.
template <class T, class Less>
SLO_SORT_HD void introsort_loop_small_(T* first, int n, int depth, Less less) {
    unsigned int st[64];
    int sp = 0;
    st[sp++] = (unsigned int)n << 13 | (unsigned int)depth << 26;
    while (sp > 0) {
        const unsigned int e = st[--sp];
        int lo = (int)(e & 0x1fffu), hi = (int)((e >> 13) & 0x1fffu), dep = (int)(e >> 26);
        while (hi - lo > 16) {
            if (dep == 0) {
                heap_sort_(first + lo, hi - lo, less);
                break;
            }
            --dep;
            T* f = first + lo;
            T* l = first + hi;
            T* mid = f + (hi - lo) / 2;
            move_median_to_first_(f, f + 1, mid, l - 1, less);
            T* cut = unguarded_partition_(f + 1, l, f, less);
            const int c = (int)(cut - first);
            st[sp++] = (unsigned int)c | (unsigned int)hi << 13 | (unsigned int)dep << 26;
            hi = c;
        }
    }
}
template <class T, class Less>
SLO_SORT_HD void std_sort_small(T* first, int n, Less less) {   // std_sort, n <= 8191
    if (n <= 1) return;
    introsort_loop_small_(first, n, 2 * lg_(n), less);
    if (n > 16) {
        insertion_sort_(first, first + 16, less);
        for (T* i = first + 16; i != first + n; ++i) unguarded_linear_insert_(i, less);
    } else {
        insertion_sort_(first, first + n, less);
    }
}
template <class T, class Less>
SLO_SORT_HD void introsort_range_small(T* first, int n, int depth, Less less) {   // introsort_range, n <= 8191
    if (n <= 1) return;
    introsort_loop_small_(first, n, depth, less);
    insertion_sort_(first, first + n, less);
}

}  // namespace slo_sort
