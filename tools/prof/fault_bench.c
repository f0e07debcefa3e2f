// Fresh-memory first-touch bandwidth with N threads, with / without MADV_HUGEPAGE (diagnostic):
// the host loader's arena columns and the report writer's buffers are fresh memory.
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
static char* buf; static size_t per; 
static void* touch(void* a) { size_t t = (size_t)a; memset(buf + t * per, 1, per); return 0; }
static double now() { struct timespec s; clock_gettime(CLOCK_MONOTONIC, &s); return s.tv_sec + s.tv_nsec / 1e9; }
int main(int argc, char** argv) {
  size_t gb = argc > 1 ? atol(argv[1]) : 8;
  int nts[] = {1, 4, 16};
  for (int huge = 0; huge < 2; huge++)
    for (int k = 0; k < 3; k++) {
      int n = nts[k]; size_t total = gb << 30; per = total / n;
      buf = mmap(0, total, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
      if (huge) madvise(buf, total, MADV_HUGEPAGE);
      double t0 = now();
      pthread_t th[64];
      for (int i = 0; i < n; i++) pthread_create(&th[i], 0, touch, (void*)(size_t)i);
      for (int i = 0; i < n; i++) pthread_join(th[i], 0);
      double dt = now() - t0;
      t0 = now();
      for (int i = 0; i < n; i++) pthread_create(&th[i], 0, touch, (void*)(size_t)i);
      for (int i = 0; i < n; i++) pthread_join(th[i], 0);
      double dt2 = now() - t0;
      printf("huge=%d threads=%2d first touch %.2f GB/s, rewrite %.2f GB/s\n", huge, n, total / dt / 1e9, total / dt2 / 1e9);
      munmap(buf, total);
    }
  FILE* f = fopen("/sys/kernel/mm/transparent_hugepage/enabled", "r");
  char s[256] = {0}; if (f) { fgets(s, sizeof s, f); fclose(f); }
  printf("THP: %s", s);
  return 0;
}
