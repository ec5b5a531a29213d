"""Literal, round-by-round restatement of the reference GPU codebook builder.

TEST INFRASTRUCTURE ONLY (see oracle/hz_oracle.c header). Pure Python, small
inputs only. It exists to pin the sequential two-queue builder in
hz_oracle.c:hzo_codebook (and the product's host builder) to the reference's
parallel algorithm, which cannot be compiled or run in this image (nvcc,
thrust and inline PTX).

Each function follows one reference function of gpuHuffmanConstruction.h; the
grid-stride loops are run serially (every thread's iteration is independent
between two Barrier::fence calls, so any serial order gives the same memory).
``F`` arithmetic wraps at ``fbits`` bits like the reference's ``unsigned int``
(fbits=32); the product uses 64-bit counts.
"""


def binary_search(freq, base, size, val):
    """gpuHuffmanConstruction.h:137-151 (BinarySearch): first index with
    freq > val, capped at size-1 (returns 0 when size <= 0)."""
    l, r = 0, size - 1
    while l < r:
        m = l + (r - l) // 2
        if freq[base + m] <= val:
            l = m + 1
        else:
            r = m
    return l


def kth_element(lf, lbase, left_size, rf, rbase, right_size, k):
    """gpuHuffmanConstruction.h:163-209 (KthElement, MERGE_PER_THREADS_1):
    position of the k-th element of the stable merge (left wins ties).
    Returns (x, y): x = left index or -1, y = right index or -1."""
    kth, li, ri = k, 0, 0
    while True:
        if left_size == li:
            return (-1, ri + kth)
        if right_size == ri:
            return (li + kth, -1)
        mid1 = li + (left_size - li) // 2
        mid2 = ri + (right_size - ri) // 2
        if mid1 - li + mid2 - ri < kth:
            if lf[lbase + mid1] > rf[rbase + mid2]:
                kth = kth - (mid2 - ri) - 1
                ri = mid2 + 1
            else:
                kth = kth - (mid1 - li) - 1
                li = mid1 + 1
        else:
            if lf[lbase + mid1] > rf[rbase + mid2]:
                left_size = mid1
            else:
                right_size = mid2


def generate_cl(hist_sorted, fbits=32):
    """gpuHuffmanConstruction.h:353-466 (GenerateCL) + 468-494 (GenerateCW) +
    551-579 (GpuCodewords::toCpu). ``hist_sorted``: the U nonzero frequencies in
    the thrust order of Compressor.cu:387-414. Returns the code strings in that
    order ('0'/'1' characters, root first), as the reference host sees them."""
    mask = (1 << fbits) - 1
    size = len(hist_sorted)
    if size == 0:
        return []
    # Node{index,left,right,parent} h:71-76, workspace h:590-615
    nodes = [[-1, -1, -1, -1] for _ in range(2 * size)]
    node_freq = [0] * size
    node_index = [0] * size
    temp_freq = [0] * size
    temp_index = [0] * size
    for i in range(size):                                  # h:365-375
        nodes[i] = [i, -1, -1, -1]
        node_freq[i] = hist_sorted[i] & mask
        node_index[i] = i
    num_current = size
    size_left = size
    while size_left > 1:                                   # h:380
        spec = (node_freq[0] + node_freq[1]) & mask        # h:381
        pivot = binary_search(node_freq, 2, size_left - 2, spec) + 2   # h:385-386
        pivot = pivot - (pivot & 1)                        # h:387
        for i in range(size_left - pivot):                 # h:390-393
            temp_freq[i] = node_freq[i + pivot]
            temp_index[i] = node_index[i + pivot]
        half = pivot >> 1
        for i in range(half):                              # h:395-426
            left = node_index[2 * i]
            right = node_index[2 * i + 1]
            nodes[left][3] = num_current + i
            nodes[right][3] = num_current + i
            nodes[num_current + i] = [-1, left, right, -1]
            temp_freq[size_left - pivot + i] = (node_freq[2 * i] + node_freq[2 * i + 1]) & mask
            temp_index[size_left - pivot + i] = num_current + i
        num_current += half                                # h:427
        ls, rs, rb = size_left - pivot, half, size_left - pivot
        new_freq = [0] * (ls + rs)
        new_index = [0] * (ls + rs)
        for i in range(ls + rs):                           # ParallelMerge h:311-324
            x, y = kth_element(temp_freq, 0, ls, temp_freq, rb, rs, i)
            if x == -1:
                new_freq[i] = temp_freq[rb + y]
                new_index[i] = temp_index[rb + y]
            else:
                new_freq[i] = temp_freq[x]
                new_index[i] = temp_index[x]
        node_freq[:ls + rs] = new_freq
        node_index[:ls + rs] = new_index
        size_left = ls + rs                                # h:441
    codes = []
    for i in range(size):                                  # GenerateCW h:468-494
        cw = []
        child, parent = i, nodes[i][3]
        while parent != -1:
            cw.append(0 if child == nodes[parent][1] else 1)
            child, parent = parent, nodes[parent][3]
        s = ''.join('1' if c == 0 else '0' for c in cw)    # toCpu h:565-572
        codes.append(s[::-1])                              # h:573
    return codes


def thrust_order(hist):
    """Compressor.cu:387-393,414,419-425: stable sort of (freq, symbol index)
    by freq, nonzero tail. Returns [(symbol, freq)]."""
    pairs = sorted(((f, s) for s, f in enumerate(hist) if f), key=lambda t: t[0])
    return [(s, f) for f, s in pairs]


def reference_codebook(hist, fbits=32):
    """{symbol: code string} and header order for a 65536-entry (or shorter)
    histogram, as Compressor.cu would build them."""
    order = thrust_order(hist)
    codes = generate_cl([f for _, f in order], fbits=fbits)
    return [s for s, _ in order], {s: c for (s, _), c in zip(order, codes)}
