# Variant patch for scripts/mkvariant.sh (run inside the copied csrc): timestamps per level in k_reduce_top
# plus an mkv_dbg_top() export. Usage: bash scripts/mkvariant.sh topdbg scripts/variants/topdbg.py; then
# MKV_LIB_PATH=abl/topdbg/lib/libmerklekv_hip.so python tools/top_dbg.py
t=open('k_reduce.hip').read()
def rep(a,b):
    global t
    assert t.count(a)==1,a[:60]; t=t.replace(a,b)
rep('''template <bool SHORT>
__global__ __launch_bounds__(RD_TILE) void k_reduce_top(TopPlan p) {''','''__device__ uint64_t g_top_dbg[64];
template <bool SHORT>
__global__ __launch_bounds__(RD_TILE) void k_reduce_top(TopPlan p) {
    if (threadIdx.x == 0 && blockIdx.x == 0) g_top_dbg[0] = __builtin_amdgcn_s_memrealtime();''')
rep('''            store_digest(p.out[k - 1] + 32 * (j - p.a[k]), o);
        }
        lds_barrier();
    }
    if (nf >= p.nl) return;''','''            store_digest(p.out[k - 1] + 32 * (j - p.a[k]), o);
        }
        lds_barrier();
        if (threadIdx.x == 0 && blockIdx.x == 0) g_top_dbg[k] = __builtin_amdgcn_s_memrealtime();
    }
    if (nf >= p.nl) return;''')
rep('''        if (!last) return;
        __threadfence();
    } else {''','''        if (!last) return;
        __threadfence();
        if (threadIdx.x == 0) { g_top_dbg[19] = blockIdx.x; g_top_dbg[20] = __builtin_amdgcn_s_memrealtime(); }
    } else {''')
rep('''            store_digest(p.out[k - 1] + 32 * i, o);
        }
        lds_barrier();
    }
}''','''            store_digest(p.out[k - 1] + 32 * i, o);
        }
        lds_barrier();
        if (threadIdx.x == 0) g_top_dbg[20 + k - nf] = __builtin_amdgcn_s_memrealtime();
    }
    if (threadIdx.x == 0) { g_top_dbg[60] = nf; g_top_dbg[61] = p.nl; g_top_dbg[62] = p.ntiles; }
}''')
t += '''
extern "C" int mkv_dbg_top(uint64_t *out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(mkv::g_top_dbg), 64 * 8) == hipSuccess ? 0 : -2;
}
'''
open('k_reduce.hip','w').write(t)
