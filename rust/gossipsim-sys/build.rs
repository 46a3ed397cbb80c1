// Link libgossipsim.so (built in-tree by `make -C dst-libp2p-test-node_amd`)
// and the HIP runtime it needs. GOSSIPSIM_LIB_DIR overrides the search path.
fn main() {
    let dir = std::env::var("GOSSIPSIM_LIB_DIR")
        .unwrap_or_else(|_| concat!(env!("CARGO_MANIFEST_DIR"), "/../../dst-libp2p-test-node_amd").to_string());
    println!("cargo:rustc-link-search=native={}", dir);
    println!("cargo:rustc-link-search=native=/opt/rocm/lib");
    println!("cargo:rustc-link-lib=dylib=gossipsim");
    println!("cargo:rustc-link-lib=dylib=amdhip64");
    println!("cargo:rerun-if-env-changed=GOSSIPSIM_LIB_DIR");
}
