# Drop-in Snappy.jl module over libsnappy_mi355x.so (see INTEGRATION.md §1).
#
# Written for the reference's Julia (REQUIRE:1 pins `julia 0.6`); the two spellings that changed
# in 0.7 (Void -> Cvoid, Vector{UInt8}(n) -> Vector{UInt8}(undef, n)) are selected by VERSION, so
# the file also loads on Julia >= 0.7.  Untested: no Julia exists in the build image or on the
# GPU box; the C ABI underneath is what the test suite exercises (tests/test_snappy_c_shape.py
# binds the same symbols with the same types).
module Snappy
export compress, uncompress

@static if VERSION < v"0.7.0-DEV"
    const VoidT = Void
    newbytes(n::Integer) = Vector{UInt8}(n)
else
    const VoidT = Cvoid
    newbytes(n::Integer) = Vector{UInt8}(undef, n)
end

const LIB = get(ENV, "SNAPPY_MI355X_LIB", "libsnappy_mi355x")
const MODES = Dict(:reference => Cint(0),  # byte-identical to Snappy.jl
                   :fast => Cint(1),       # wave-parallel parse; decodes bit-exactly under Snappy.jl
                   :dense => Cint(2))      # :fast verifying two chain candidates: smaller output
const CTX = Ref{Ptr{VoidT}}(C_NULL)

function __init__()
    CTX[] = ccall((:sm_ctx_create, LIB), Ptr{VoidT}, (Cint,), 0)
    CTX[] == C_NULL && error("no usable MI355X device")
end

status_message(st) = unsafe_string(ccall((:sm_status_message, LIB), Cstring, (Cint,), st))

maxlength_compressed(n::Integer) = Int(ccall((:sm_max_compressed_length, LIB), Csize_t, (Csize_t,), n))

# src/Snappy.jl:20.  mode=:dense (default) is the GPU's wave-parallel parse checking two chain
# candidates: its streams decode bit-exactly under Snappy.jl's uncompress (the reference's tests
# pin round trips, not bytes) and are within 1.01x of Snappy.jl's size on every corpus file, at a
# single call's cost; :fast is the batch default (up to 1.04x); :reference returns Snappy.jl's
# exact bytes.
function compress(input::Vector{UInt8}; mode::Symbol=:dense)
    length(input) > typemax(UInt32) && error("Input too large.")
    output = newbytes(maxlength_compressed(length(input)))
    outlen = Ref{Csize_t}(length(output))
    st = ccall((:sm_compress, LIB), Cint,
               (Ptr{VoidT}, Ptr{UInt8}, Csize_t, Ptr{UInt8}, Ref{Csize_t}, Cint),
               CTX[], input, length(input), output, outlen, MODES[mode])
    st == 0 || error(status_message(st))
    return resize!(output, outlen[])
end
compress(input::String; mode::Symbol=:dense) = compress(Vector{UInt8}(input); mode=mode)  # src/Snappy.jl:38

function length_uncompressed(input::Vector{UInt8})  # src/Snappy.jl:90 (1-based next index)
    v = Ref{UInt32}(0); nx = Ref{Csize_t}(0)
    st = ccall((:sm_parse32, LIB), Cint, (Ptr{UInt8}, Csize_t, Csize_t, Ref{UInt32}, Ref{Csize_t}),
               input, length(input), 0, v, nx)
    st == 0 || error(status_message(st))
    return (v[], Int(nx[]) + 1)
end

function uncompress(input::Vector{UInt8})           # src/Snappy.jl:46
    n, _ = length_uncompressed(input)
    output = newbytes(n)
    outlen = Ref{Csize_t}(n)
    st = ccall((:sm_uncompress, LIB), Cint,
               (Ptr{VoidT}, Ptr{UInt8}, Csize_t, Ptr{UInt8}, Ref{Csize_t}),
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
    tmp = newbytes(5)
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

# test/libsnappy.jl:5-30's ccall signatures, rebound by library and symbol name alone: the
# ctx-less snappy-c.h-shaped entry points (a default context on device $SNAPPY_MI355X_DEVICE,
# SM_MODE_FAST_DENSE unless sm_snappy_set_mode says otherwise).
function gpu_compress(src::Vector{UInt8})
    cap = ccall((:sm_snappy_max_compressed_length, LIB), Csize_t, (Csize_t,), length(src))
    dst = newbytes(cap)
    len = Ref{Csize_t}(cap)
    st = ccall((:sm_snappy_compress, LIB), Cint, (Ptr{UInt8}, Csize_t, Ptr{UInt8}, Ref{Csize_t}),
               src, length(src), dst, len)
    st == 0 || error(status_message(st))
    return resize!(dst, len[])
end

function gpu_uncompress(src::Array{UInt8})
    len = Ref{Csize_t}(0)
    st = ccall((:sm_snappy_uncompressed_length, LIB), Cint, (Ptr{UInt8}, Csize_t, Ref{Csize_t}),
               src, length(src), len)
    st == 0 || error(status_message(st))
    dst = newbytes(len[])
    st = ccall((:sm_snappy_uncompress, LIB), Cint, (Ptr{UInt8}, Csize_t, Ptr{UInt8}, Ref{Csize_t}),
               src, length(src), dst, len)
    st == 0 || error(status_message(st))
    return dst
end
end
