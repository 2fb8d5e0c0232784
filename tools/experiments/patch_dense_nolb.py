# Timing-only ablation of k_parse_dense: the store wave takes a fixed per-tile offset (t x tile
# frames) instead of the decoupled look-back -- the output is NOT the dense order; it measures what
# the kernel costs without the cross-block dependency.
if f == "fb_parse.hip":
    a = "            unsigned long long excl = 0ull;\n            if (t == 0u) {"
    assert a in s
    s = s.replace(a, "            unsigned long long excl = (unsigned long long)(t * kDnTileSegs * 64u) | ((unsigned long long)(t * kDnTileSegs * 64u) << 32);\n            if (false) {", 1)
