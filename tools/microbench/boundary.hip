// Kernel-boundary cost on MI355X: back-to-back launches on one stream, a writer of `mb` MB (plain,
// nontemporal or sc1 stores) followed by a small reader, per iteration wall time by hipEvents.
// Tells whether the LocalBA trial chain's inter-launch gaps (~3.5 us each) come from the L2
// write-back of the records a kernel leaves dirty.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int MODE> __global__ void writer(double *p, size_t n, double v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        if (MODE == 0) p[i] = v + i;
        else if (MODE == 1) __builtin_nontemporal_store(v + i, p + i);
        else __hip_atomic_store((unsigned long long *)(p + i), (unsigned long long)(v + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
__global__ void reader(const double *p, double *o) {
    double s = 0;
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) s += p[i * 97];
    if (s == 12345.0) o[0] = s;
}
__global__ void empty(double *o) { if (o[0] == 12345.0) o[1] = 1; }
int main() {
    hipStream_t st; (void)hipStreamCreate(&st);
    double *p, *o; (void)hipMalloc(&p, 64 << 20); (void)hipMalloc(&o, 64); (void)hipMemset(o, 0, 64);
    hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    const int IT = 300;
    auto run = [&](const char *name, auto &&body) {
        for (int w = 0; w < 20; w++) body();
        (void)hipStreamSynchronize(st);
        (void)hipEventRecord(a, st);
        for (int i = 0; i < IT; i++) body();
        (void)hipEventRecord(b, st);
        (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b);
        printf("%-44s %.2f us / iteration\n", name, 1000.0 * ms / IT);
    };
    run("empty", [&] { empty<<<1, 64, 0, st>>>(o); });
    {   // the same chains captured in a graph: GPU-side dispatch cost without the host enqueue
        auto graph_run = [&](const char *name, int per, auto &&body) {
            hipGraph_t gr; hipGraphExec_t ge;
            (void)hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
            for (int i = 0; i < IT; i++) body();
            (void)hipStreamEndCapture(st, &gr);
            (void)hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0);
            (void)hipGraphLaunch(ge, st); (void)hipStreamSynchronize(st);
            (void)hipEventRecord(a, st);
            (void)hipGraphLaunch(ge, st);
            (void)hipEventRecord(b, st);
            (void)hipEventSynchronize(b);
            float ms; (void)hipEventElapsedTime(&ms, a, b);
            printf("%-44s %.2f us / iteration (%d kernels)\n", name, 1000.0 * ms / IT, per);
            (void)hipGraphExecDestroy(ge); (void)hipGraphDestroy(gr);
        };
        graph_run("graph: empty", 1, [&] { empty<<<1, 64, 0, st>>>(o); });
        const size_t n7 = (size_t)7 * (1 << 20) / 8;
        graph_run("graph: write 7 MB plain + reader", 2, [&] { writer<0><<<1024, 256, 0, st>>>(p, n7, 1.0); reader<<<1, 256, 0, st>>>(p, o); });
        graph_run("graph: write 7 MB sc1 + reader", 2, [&] { writer<2><<<1024, 256, 0, st>>>(p, n7, 1.0); reader<<<1, 256, 0, st>>>(p, o); });
    }
    run("empty x2", [&] { empty<<<1, 64, 0, st>>>(o); empty<<<1, 64, 0, st>>>(o); });
    for (int mb : {1, 7, 28}) {
        const size_t n = (size_t)mb * (1 << 20) / 8;
        char nm[64];
        snprintf(nm, 64, "write %d MB plain", mb);
        run(nm, [&] { writer<0><<<1024, 256, 0, st>>>(p, n, 1.0); });
        snprintf(nm, 64, "write %d MB plain + reader", mb);
        run(nm, [&] { writer<0><<<1024, 256, 0, st>>>(p, n, 1.0); reader<<<1, 256, 0, st>>>(p, o); });
        snprintf(nm, 64, "write %d MB nontemporal + reader", mb);
        run(nm, [&] { writer<1><<<1024, 256, 0, st>>>(p, n, 1.0); reader<<<1, 256, 0, st>>>(p, o); });
        snprintf(nm, 64, "write %d MB sc1 + reader", mb);
        run(nm, [&] { writer<2><<<1024, 256, 0, st>>>(p, n, 1.0); reader<<<1, 256, 0, st>>>(p, o); });
        snprintf(nm, 64, "write %d MB plain + reader + reader", mb);
        run(nm, [&] { writer<0><<<1024, 256, 0, st>>>(p, n, 1.0); reader<<<1, 256, 0, st>>>(p, o); reader<<<1, 256, 0, st>>>(p, o); });
    }
    return 0;
}
