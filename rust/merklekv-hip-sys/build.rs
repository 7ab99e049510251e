// Link libmerklekv_hip.so (built by `make -C merklekv_amd/csrc`, HIP for gfx950). MERKLEKV_HIP_LIB_DIR
// overrides the default: the repository's merklekv_amd/lib next to this crate.
use std::env;
use std::path::PathBuf;

fn main() {
    let dir = env::var("MERKLEKV_HIP_LIB_DIR").map(PathBuf::from).unwrap_or_else(|_| {
        PathBuf::from(env::var("CARGO_MANIFEST_DIR").unwrap()).join("../../merklekv_amd/lib")
    });
    println!("cargo:rustc-link-search=native={}", dir.display());
    println!("cargo:rustc-link-lib=dylib=merklekv_hip");
    // the shared library finds itself at run time without LD_LIBRARY_PATH
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", dir.display());
    println!("cargo:rerun-if-env-changed=MERKLEKV_HIP_LIB_DIR");
    println!("cargo:rerun-if-changed=../../include/mkv_merkle.h");
}
