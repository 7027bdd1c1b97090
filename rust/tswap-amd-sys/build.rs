// Link against libtswap_hip.so (built by __graft_entry__.build() into p2p_distributed_tswap_amd/).
// TSWAP_AMD_LIB_DIR: directory holding the library; the ROCm runtime it needs (libamdhip64) is
// found through the usual loader path (/opt/rocm/lib).
fn main() {
    let dir = std::env::var("TSWAP_AMD_LIB_DIR")
        .unwrap_or_else(|_| "../../p2p_distributed_tswap_amd".to_string());
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=tswap_hip");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{dir}");
    println!("cargo:rerun-if-env-changed=TSWAP_AMD_LIB_DIR");
}
