## R front-end of the MI355X k-mer position index.
## Same three functions, arguments and results as the reference's index API
## (reference kmer_hash.R:5-28); only the shared object changes: kmer_hash.so is built from
## kmer_hash_glue.c over libkmhgpu.so (see INTEGRATION.md).
local({
    here <- dirname(sys.frame(1)$ofile)
    dyn.load(file.path(here, "kmer_hash.so"))
})

## build the index; positions come back ascending per k-mer whatever do.sort says
make.kmer.hash <- function(seq, k, do.sort=FALSE){
    .Call("make_kmer_h_index", as.character(seq), as.integer(k), as.integer(do.sort))
}

## opt.flag bits: 1 k-mer strings, 2 (i, pos) rows, 4 (i, x, y) pair rows, 8 counts
kmer.pos <- function(ex.ptr, opt.flag){
    res <- .Call("kmer_positions", ex.ptr, as.integer(opt.flag))
    if(!is.null(res$pos)){
        res$pos <- t(res$pos)
        colnames(res$pos) <- c("i", "pos")
    }
    if(!is.null(res$pair.pos)){
        res$pair.pos <- t(res$pair.pos)
        colnames(res$pair.pos) <- c("i", "x", "y")
    }
    res
}

## dot-plot rows: i = end of the query window, j = start of the indexed occurrence
seq.kmer.pos <- function(ex.ptr, seq, k){
    m <- .Call("sequence_kmer_positions", ex.ptr, as.character(seq), as.integer(k))
    rownames(m) <- c("i", "j")
    t(m)
}

## shared k-mers of two indices: rows (a, b) = a position in ptr.a with a position in ptr.b
## (the reference's version crashes, test.R:330; this one visits only live k-mers, same k)
kmer.pairs <- function(ptr.a, ptr.b){
    tmp <- t(.Call("kmer_pair_pos", ptr.a, ptr.b))
    colnames(tmp) <- c("a", "b")
    tmp
}

## per-source k-mer counts; params = c(k, source, source_n); kmer.pos / seq.kmer.pos read the
## count vectors of the returned pointer as positions (reference kmer_hash.R:43-46)
count.kmers <- function(seq, params, hash.ptr=NULL){
    params <- as.integer(params)
    .Call("count_kmers", hash.ptr, params, seq)
}

## not in the reference: kmer.pos k-mer order, "first" (default) or "khash" (the reference's
## bucket order: byte-identical kmer.pos output)
kmer.row.order <- function(ex.ptr, order="khash"){
    invisible(.Call("kmer_row_order", ex.ptr, as.character(order)))
}

## canonical k-mer counts of a FASTA/FASTQ file (plain or gzip) into a suffix_hash_n pointer;
## params = c(k, prefix_bits, min_q, thread_n, max_reads, max_mem, source_n, source)
## (reference kmer_hash.R:70-73; counted on the GPU, prefix_bits / thread_n / max_mem only
## change the reference's memory layout and threading, not the counts)
count.kmers.fq.sh.rp <- function(fq.file, params, hash.ptr=NULL){
    params <- as.integer(params)
    .Call("count_kmers_fastq_sh_rp", hash.ptr, params, fq.file)
}

## counts_n x nchar(seq) matrix of canonical k-mer counts along seq (reference kmer_hash.R:75-78)
seq.kmer.depth.sh <- function(hash.ptr, seq, k){
    .Call("seq_kmer_depth_sh", hash.ptr, as.character(seq), as.integer(k))
}

## k-mer count spectra per source combination (reference kmer_hash.R:88-91)
kmer.spec.sh.n <- function(ptr, max.count, comb, comb.inner, source.min){
    .Call("kmer_spectrum_suffix_hash_n", ptr, as.integer(max.count),
          as.integer(comb), as.integer(comb.inner), as.integer(source.min))
}
