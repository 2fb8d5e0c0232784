# Timing-only ablation of k_parse_dense (tools/build_variants.sh PATCH): the store wave takes a fixed
# per-tile offset (t x tile frames, for records and DNS records alike) and skips the decoupled
# look-back entirely -- the output is NOT the dense order; it measures what the kernel costs without
# the cross-block dependency.  (Round 4's version kept the look-back in the else branch and so ADDED
# the real prefix to the fixed offset, writing past the batch: the illegal access in
# gpurun_out/r4dn/nolb.1.err, DESIGN §3.2 "Bounded copies".  The status-word store of tile 0 is
# dropped too: taken by every tile, 4,096 stores to one address cost 50.6 vs 38.5 us per batch.)
if f == "fb_parse.hip":
    a = "            unsigned long long excl = 0ull;\n            if (t == 0u) {"
    assert a in s
    s = s.replace(a, "            unsigned long long excl = (unsigned long long)(t * kDnTileSegs * 64u) | ((unsigned long long)(t * kDnTileSegs * 64u) << 32);\n            if (true) {", 1)
    b = "                if (lane == 0u) __hip_atomic_store(P.dstatus, dn_word(ep, kDnP, agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);\n"
    assert b in s
    s = s.replace(b, "", 1)
