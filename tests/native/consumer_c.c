/* consumer_c.c — TEST HARNESS: the boundary used from strict C99 (gcc -std=c99 -pedantic), the way a
 * cgo / FFI binding or a C node would: compile-and-link check of include/llsr.h against libllsr.so
 * (tests/test_abi.py). Not run: it only has to build. */
#include <stdio.h>

#include "llsr.h"

int main(void) {
  llsr_config cfg;
  llsr_handle* h = NULL;
  llsr_sizes sz;
  llsr_scan_out out;
  llsr_lm_report rep;
  llsr_s2s_report srep;
  float pose[6] = {0, 0, 0, 0, 0, 0};
  float tc[6] = {0, 0, 0, 0, 0, 0};
  int32_t deg = 0;
  int32_t rc = llsr_abi_version() == LLSR_ABI_VERSION ? LLSR_OK : LLSR_EINVAL;
  if (rc == LLSR_OK) rc = llsr_config_default(&cfg, LLSR_LIDAR_VLP16);
  if (rc == LLSR_OK) rc = llsr_create(&cfg, 0, 1, 30000, &h);
  if (rc != LLSR_OK) {
    printf("llsr_create: %d\n", (int)rc);
    return 1;
  }
  llsr_query_sizes(h, &sz);
  out.n_points = 0;
  rc = llsr_process_scan(h, NULL, 0, &out);
  rc = llsr_scan2scan(h, NULL, 0, NULL, 0, NULL, 0, NULL, 0, tc, &deg, &srep);
  rc = llsr_scan2map(h, NULL, 0, NULL, 0, NULL, 0, NULL, 0, pose, &rep);
  llsr_destroy(h);
  return rc == LLSR_OK ? 0 : 1;
}
