// pt_sweep_all.hip — the A/B instance of the PT sweep kernel (pt_sweep.hip with ALL = true): every PQD_PT_MODE,
// the 4M column products and the 16x16 column tiles at N2 not a multiple of 16. Selected by the host when a switch
// asks for a non-default variant (SweepParams::variants); the default path runs pt_sweep.hip's production instance.
#define PQD_SWEEP_ALL_TU 1
#include "pt_sweep.hip"
