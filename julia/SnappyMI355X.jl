# Drop-in Snappy.jl module over libsnappy_mi355x.so (see INTEGRATION.md). Untested here:
# Julia is not installed in the build image.
module Snappy
export compress, uncompress

const LIB = get(ENV, "SNAPPY_MI355X_LIB", "libsnappy_mi355x")
const SM_MODE_REFERENCE = Cint(0)      # byte-identical to Snappy.jl
const SM_MODE_FAST = Cint(1)           # wave-parallel parse; decodes bit-exactly under Snappy.jl
const SM_MODE_FAST_DENSE = Cint(2)     # SM_MODE_FAST with two chain candidates: smaller output
const CTX = Ref{Ptr{Cvoid}}(C_NULL)

function __init__()
    CTX[] = ccall((:sm_ctx_create, LIB), Ptr{Cvoid}, (Cint,), 0)
    CTX[] == C_NULL && error("no usable MI355X device")
end

status_message(st) = unsafe_string(ccall((:sm_status_message, LIB), Cstring, (Cint,), st))

maxlength_compressed(n::Integer) = Int(ccall((:sm_max_compressed_length, LIB), Csize_t, (Csize_t,), n))

function compress(input::Vector{UInt8})            # src/Snappy.jl:20
    length(input) > typemax(UInt32) && error("Input too large.")
    output = Vector{UInt8}(undef, maxlength_compressed(length(input)))
    outlen = Ref{Csize_t}(length(output))
    st = ccall((:sm_compress, LIB), Cint,
               (Ptr{Cvoid}, Ptr{UInt8}, Csize_t, Ptr{UInt8}, Ref{Csize_t}, Cint),
               CTX[], input, length(input), output, outlen, SM_MODE_REFERENCE)
    st == 0 || error(status_message(st))
    return resize!(output, outlen[])
end
compress(input::String) = compress(Vector{UInt8}(input))   # src/Snappy.jl:38

function length_uncompressed(input::Vector{UInt8})  # src/Snappy.jl:90 (1-based next index)
    v = Ref{UInt32}(0); nx = Ref{Csize_t}(0)
    st = ccall((:sm_parse32, LIB), Cint, (Ptr{UInt8}, Csize_t, Csize_t, Ref{UInt32}, Ref{Csize_t}),
               input, length(input), 0, v, nx)
    st == 0 || error(status_message(st))
    return (v[], Int(nx[]) + 1)
end

function uncompress(input::Vector{UInt8})           # src/Snappy.jl:46
    n, _ = length_uncompressed(input)
    output = Vector{UInt8}(undef, n)
    outlen = Ref{Csize_t}(n)
    st = ccall((:sm_uncompress, LIB), Cint,
               (Ptr{Cvoid}, Ptr{UInt8}, Csize_t, Ptr{UInt8}, Ref{Csize_t}),
               CTX[], input, length(input), output, outlen)
    st == 0 || error(status_message(st))            # the reference's exact message text
    return output
end

# helpers the reference's own tests call (test/runtests.jl:96-173), 1-based like the reference
function parse32(buf::Vector{UInt8}, offset::Integer)                 # src/varint.jl:12
    v = Ref{UInt32}(0); nx = Ref{Csize_t}(0)
    st = ccall((:sm_parse32, LIB), Cint, (Ptr{UInt8}, Csize_t, Csize_t, Ref{UInt32}, Ref{Csize_t}),
               buf, length(buf), offset - 1, v, nx)
    st == 0 || error(status_message(st))
    return (v[], Int(nx[]) + 1)
end
function encode32!(buf::Vector{UInt8}, offset::Integer, value::UInt32)  # src/varint.jl:46
    tmp = Vector{UInt8}(undef, 5)
    n = ccall((:sm_encode32, LIB), Csize_t, (Ptr{UInt8}, UInt32), tmp, value)
    buf[offset:offset+n-1] = tmp[1:n]
    return offset + n
end
function find_match_length(a::Vector{UInt8}, i1::Integer, i2::Integer, limit::Integer)  # internal.jl:343
    m = Ref{Csize_t}(0)
    st = ccall((:sm_find_match_length, LIB), Cint, (Ptr{UInt8}, Csize_t, Csize_t, Csize_t, Csize_t, Ref{Csize_t}),
               a, length(a), i1 - 1, i2 - 1, limit - 1, m)
    st == 0 || throw(BoundsError(a, limit))   # the reference reads past `a` here (@test_broken)
    return Int(m[])
end
end
