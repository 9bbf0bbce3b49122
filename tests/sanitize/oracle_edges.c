/* Host-only sanitizer driver for the oracle restatement: edge shapes the
 * reference mishandles (k > frames, one frame, 64 channels, k = 1). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

int oracle_mavg_i16(const int16_t*, int16_t*, size_t, int, int);
int oracle_mavg_f32(const float*, float*, size_t, int, int);
int oracle_mavg_f32_mt(const float*, float*, size_t, int, int, int);
int oracle_window_sum_i64(const int16_t*, size_t, int, int, size_t, size_t, int64_t*);

int main(void) {
    const int shapes[][3] = {{1, 1, 1}, {1, 1, 5}, {3, 2, 7}, {64, 64, 3}, {100, 1, 1000}, {257, 4, 256}, {0, 1, 3}};
    for (unsigned s = 0; s < sizeof shapes / sizeof shapes[0]; ++s) {
        const size_t frames = (size_t)shapes[s][0];
        const int C = shapes[s][1], k = shapes[s][2];
        const size_t n = frames * (size_t)C;
        int16_t* x = malloc((n ? n : 1) * sizeof *x);
        int16_t* y = malloc((n ? n : 1) * sizeof *y);
        float* xf = malloc((n ? n : 1) * sizeof *xf);
        float* yf = malloc((n ? n : 1) * sizeof *yf);
        int64_t* w = malloc((n ? n : 1) * sizeof *w);
        for (size_t i = 0; i < n; ++i) { x[i] = (int16_t)(i * 7919u); xf[i] = (float)x[i]; }
        if (oracle_mavg_i16(x, y, n, C, k) || oracle_mavg_f32(xf, yf, n, C, k) ||
            oracle_mavg_f32_mt(xf, yf, n, C, k, 3) || oracle_window_sum_i64(x, n, C, k, 0, frames, w)) {
            printf("unexpected error at shape %u\n", s);
            return 1;
        }
        free(x); free(y); free(xf); free(yf); free(w);
    }
    printf("edges ok\n");
    return 0;
}
