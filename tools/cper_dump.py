#!/usr/bin/env python3
"""amd-smi CPER (RAS error record) query on every GPU: status, entry count and severities (non-root)."""
import json

import amdsmi as A

A.amdsmi_init()
out = []
for i, h in enumerate(A.amdsmi_get_processor_handles()):
    row = {"gpu": i}
    for name, mask in (("all", 0x7), ("fatal", 1 << 1), ("uncorrected", 1 << 0), ("corrected", 1 << 2)):
        try:
            entries, cursor, hdrs, status = A.amdsmi_get_gpu_cper_entries(h, mask)
            row[name] = {"entries": len(hdrs) if isinstance(hdrs, list) else hdrs, "cursor": cursor, "status": status,
                         "first": (hdrs[0] if isinstance(hdrs, list) and hdrs else None)}
        except Exception as e:
            row[name] = repr(e)
    out.append(row)
print(json.dumps(out, default=str, indent=1))
