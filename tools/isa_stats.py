"""Instruction-mix summary of one kernel in a device assembly file
(hipcc --cuda-device-only -S).  usage: isa_stats.py file.s [kernel-substring]"""
import re
import sys

text = open(sys.argv[1]).read()
key = sys.argv[2] if len(sys.argv) > 2 else "be_kernelILi10ELi0E"
m = re.search(r"^(\S*%s\S*):" % re.escape(key), text, re.M)
body = text[m.end():text.index(".Lfunc_end", m.end())]
ins = [l.split()[0] for l in body.splitlines() if l.startswith("\t") and not l.strip().startswith((";", "."))]
count = lambda p: sum(1 for i in ins if i.startswith(p))
print(m.group(1), {"instr": len(ins), "s_cbranch": count("s_cbranch"), "execz": count("s_cbranch_execz"),
      "saveexec": sum("saveexec" in i for i in ins), "s_nop": count("s_nop"), "readlane": count("v_readlane"),
      "writelane": count("v_writelane"), "global_load": count("global_load"), "global_store": count("global_store"),
      "ds": count("ds_"), "v_mul_f64": count("v_mul_f64") + count("v_fma_f64"), "s_waitcnt": count("s_waitcnt")})
