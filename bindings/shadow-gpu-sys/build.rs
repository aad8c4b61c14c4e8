// Link libshadow_gpu.so: SHADOW_GPU_LIB_DIR names the directory holding it (the
// shadow_amd/ directory of a built tree); otherwise the system search path is used.
fn main() {
    println!("cargo:rerun-if-env-changed=SHADOW_GPU_LIB_DIR");
    if let Ok(dir) = std::env::var("SHADOW_GPU_LIB_DIR") {
        println!("cargo:rustc-link-search=native={dir}");
    }
    println!("cargo:rustc-link-lib=dylib=shadow_gpu");
}
