if f == "fb_flow.hip":
    R = []
    R.append(("    for (uint32_t h = blockIdx.x; h < n_hot; h += gridDim.x) {\n", "    unsigned long long kt[5] = {0ull, 0ull, 0ull, 0ull, 0ull}; uint32_t kg = 0u, kr = 0u; unsigned long long kc = wall_clock64();\n#define KT(i) { const unsigned long long t_ = wall_clock64(); kt[i] += t_ - kc; kc = t_; }\n    for (uint32_t h = blockIdx.x; h < n_hot; h += gridDim.x) {\n        KT(4)\n"))
    R.append(("        const uint32_t row = *rowp, cnt = row >> 16;\n", "        const uint32_t row = *rowp, cnt = row >> 16;\n        ++kg; kr += cnt;\n"))
    R.append(("        // reduce per key (a key the table cannot take stays a plain entry)\n", "        KT(0)\n        // reduce per key (a key the table cannot take stays a plain entry)\n"))
    R.append(("        // number the keys met more than once; one global atomic per group for their ids\n", "        KT(1)\n        // number the keys met more than once; one global atomic per group for their ids\n"))
    R.append(("        {   // the order bitmap", "        KT(2)\n        {   // the order bitmap"))
    R.append(("        // the combined entries (two units each in P.comb) and their index words behind the kept ones\n", "        KT(3)\n        // the combined entries (two units each in P.comb) and their index words behind the kept ones\n"))
    R.append(("        __syncthreads();  // the table is re-initialised for the next group\n    }\n}\n", "        __syncthreads();  // the table is re-initialised for the next group\n    }\n    KT(4)\n    if (threadIdx.x == 0 && blockIdx.x % 37u == 0u) printf(\"CP wg %u groups %u recs %u init %llu reduce %llu ids %llu pack %llu rest %llu\\n\", blockIdx.x, kg, kr, kt[0], kt[1], kt[2], kt[3], kt[4]);\n}\n"))
    for a, b in R:
        assert a in s, a
        s = s.replace(a, b, 1)
