# A/B (round 6): the thread id made opaque at the top of every island iteration and every TOI pass
# (an empty asm with an in/out operand), so LDS addresses derived from it are made inside those loops
# instead of being hoisted to the kernel's entry and held across the step (v0's k_step spilled 14 of
# them to scratch at entry: 13.6 MB of scratch writes per 4096-lane launch).
EDITS = [
    ("mrp_world.h", "    const int tid;\n    int step_prio", "    int tid;             // made opaque per island / TOI pass by refresh_tid (MRP_FRESH_REGS)\n    int step_prio"),
    ("mrp_world.h", "    // ------------------------------------------------------------------ bodies\n",
     """    // MRP_FRESH_REGS: a copy of tid the compiler cannot prove equal to the one before it, so the LDS
    // addresses derived from it are made inside the loop that refreshes it, not hoisted to k_step's
    // entry and kept (or spilled) across the whole step
    __device__ __forceinline__ void refresh_tid() {
#if MRP_FRESH_REGS
        asm volatile("" : "+v"(tid));
#endif
    }

    // ------------------------------------------------------------------ bodies
"""),
    ("mrp_world.h", "            MRP_PROG(0x3000u + nisl);\n", "            MRP_PROG(0x3000u + nisl);\n            refresh_tid();\n"),
    ("mrp_world.h", "            MRP_PROG(0x2000u + pass);\n", "            MRP_PROG(0x2000u + pass);\n            refresh_tid();\n"),
]
