// Phase timestamps of the ELBO-finishing launches (MI_FINISH_TIMING builds only,
// tools/finish_timing.py): thread 0 of every block writes the wall clock (100 MHz) at up to eight
// points into a buffer set by mi_*_finish_timing. Compiled out otherwise.
#pragma once

#ifndef MI_FINISH_TIMING
#define MI_FINISH_TIMING 0
#endif

#if MI_FINISH_TIMING
#define MI_FIN_STAMP(buf, i)                                                         \
  do {                                                                               \
    if (threadIdx.x == 0 && (buf) != nullptr) (buf)[(int64_t)blockIdx.x * 8 + (i)] = \
        wall_clock64();                                                              \
  } while (0)
#else
#define MI_FIN_STAMP(buf, i) do { } while (0)
#endif
