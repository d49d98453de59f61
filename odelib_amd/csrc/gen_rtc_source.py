"""Embed ode_kernels.cuh as a C++ raw string for the hipRTC path (build step)."""
import sys

import os

src = open(sys.argv[1]).read()
here = os.path.dirname(os.path.abspath(sys.argv[1]))
keep = []


def add(text):
    for line in text.splitlines():
        s = line.strip()
        if s.startswith('#include "') and s != '#include "models.cuh"':
            add(open(os.path.join(here, s.split('"')[1])).read())  # our own headers: inline
            continue
        if s.startswith("#include") or s == "#pragma once" or s.startswith("//"):
            continue  # system includes are provided by hipRTC; comments are not needed at run time
        keep.append(line)


add(src)
body = "\n".join(keep)
assert ")OE_RTC\"" not in body
with open(sys.argv[2], "w") as f:
    f.write("// generated from ode_kernels.cuh by gen_rtc_source.py — do not edit\n")
    f.write('static const char* kRtcKernelSource = R"OE_RTC(\n' + body + '\n)OE_RTC";\n')
