#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
int main() {
    void* d; hipMalloc(&d, 1 << 20);
    char* m = (char*)malloc(1 << 26); m[0] = 1;
    void* h; hipHostMalloc(&h, 1 << 20, 0);
    void* ptrs[3] = {m, h, d};
    const char* names[3] = {"malloc", "hipHostMalloc", "hipMalloc"};
    for (int i = 0; i < 3; i++) {
        hipPointerAttribute_t a; memset(&a, 0, sizeof(a));
        hipError_t e = hipPointerGetAttributes(&a, ptrs[i]);
        printf("%s: err=%d type=%d\n", names[i], (int)e, (int)a.type);
        (void)hipGetLastError();
    }
}
