"""Embed ode_kernels.cuh as a C++ raw string for the hipRTC path (build step)."""
import sys

src = open(sys.argv[1]).read()
keep = []
for line in src.splitlines():
    s = line.strip()
    if s.startswith("#include") or s == "#pragma once" or s.startswith("//"):
        continue  # includes are provided by hipRTC; comments are not needed at run time
    keep.append(line)
body = "\n".join(keep)
assert ")OE_RTC\"" not in body
with open(sys.argv[2], "w") as f:
    f.write("// generated from ode_kernels.cuh by gen_rtc_source.py — do not edit\n")
    f.write('static const char* kRtcKernelSource = R"OE_RTC(\n' + body + '\n)OE_RTC";\n')
