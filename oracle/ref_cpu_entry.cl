/*
 * ref_cpu_entry.cl -- the UNMODIFIED reference kernel, #included in place (nothing copied or
 * edited) for the x86-64 build of `make -C oracle refcpu` (test infrastructure; see
 * ref_cpu_host.c).
 */
#include "kernel_bvh.cl"
