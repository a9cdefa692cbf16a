/* Prints sizeof / offsetof of the ABI structs; tests/test_abi.py compares them
 * with the ctypes mirror in hstream_amd/abi.py. */
#include <stddef.h>
#include <stdio.h>
#include "../include/hstream_gpu.h"
#include "../include/hstream_ingest.h"
#include "../include/hstream_sink.h"
#include "../include/hstream_join.h"
#define F(T, m) printf("%s.%s %zu\n", #T, #m, offsetof(T, m))
#define S(T) printf("%s %zu\n", #T, sizeof(T))
int main(void) {
  S(hsg_engine_config); F(hsg_engine_config, comm_id); F(hsg_engine_config, batch_capacity);
  S(hsg_agg);
  S(hsg_op_config); F(hsg_op_config, size_ms); F(hsg_op_config, grace_ms); F(hsg_op_config, n_cols);
  F(hsg_op_config, col_types); F(hsg_op_config, aggs); F(hsg_op_config, state_capacity); F(hsg_op_config, out_capacity); F(hsg_op_config, flags);
  S(hsg_batch); F(hsg_batch, key_id); F(hsg_batch, ts); F(hsg_batch, cols); F(hsg_batch, valid); F(hsg_batch, ready_event); F(hsg_batch, key_enc); F(hsg_batch, ts_base); F(hsg_batch, col_enc); F(hsg_batch, col_scale); F(hsg_batch, ts_frames);
  S(hsg_rows); F(hsg_rows, key_id); F(hsg_rows, win_start); F(hsg_rows, src_index); F(hsg_rows, aggs); F(hsg_rows, form);
  S(hsg_stats); F(hsg_stats, last_batch_ms); F(hsg_stats, exchange_bytes); F(hsg_stats, touched_total); F(hsg_stats, state_row_bytes); F(hsg_stats, spill_events); F(hsg_stats, grow_events); F(hsg_stats, replays); F(hsg_stats, overflow_rebuilds);
  S(hsg_decoder_config); F(hsg_decoder_config, n_cols); F(hsg_decoder_config, col_fields); F(hsg_decoder_config, col_numeric); F(hsg_decoder_config, literal_forms);
  S(hsg_decode_buffers); F(hsg_decode_buffers, ts_frames); F(hsg_decode_buffers, valid); F(hsg_decode_buffers, allow); F(hsg_decode_buffers, col_ptrs); F(hsg_decode_buffers, valid_ptrs);
  S(hsg_sink_config); F(hsg_sink_config, key_field); F(hsg_sink_config, agg_index);
  S(hsg_sink_records); F(hsg_sink_records, key_capacity); F(hsg_sink_records, key_bytes); F(hsg_sink_records, value_off);
  S(hsg_sink_spellings); F(hsg_sink_spellings, n); F(hsg_sink_spellings, src_base); F(hsg_sink_spellings, mem);
  S(hsg_join_config); F(hsg_join_config, batch_capacity);
  S(hsg_join_batch); F(hsg_join_batch, side); F(hsg_join_batch, handle);
  S(hsg_join_rows); F(hsg_join_rows, this_handle); F(hsg_join_rows, ts);
  return 0;
}
